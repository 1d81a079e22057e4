set -o pipefail
V=is3d2_amd/variants
# round 6 r6j: bisect the F_TS slowdown against the round-5 final build (r5final = d6c93a5): v_cd77 = cd77dd5 (bench launch,
# deterministic split count, k_fold gate), v_a109 = a1099a0 (modified table-only tiles, float divmod), fdiv0 = HEAD with
# IS3D_TAB_FDIV=0, default = HEAD (modified launches without {b', Phi} rows)
timeout -k 10 400 tools/ab.sh config4 "2" default $V/r5final.so $V/v_cd77.so $V/v_a109.so $V/fdiv0.so && \
timeout -k 10 300 tools/ab.sh config2 "1 2" default $V/r5final.so $V/v_cd77.so $V/v_a109.so $V/fdiv0.so
