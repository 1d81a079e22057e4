"""Pack the reference's own test configurations, tests/modified_distribution/ of xyw2016/iS3D2
(64 iS3D_parameters.dat variants over {central, noncentral} x {small, large}_bulk
x {grad, ce, ptm, ptb} x {none, shear, bulk, shear_bulk}, their pT / phi / y / eta tables and the
3-species chosen list), into tests/golden/modified_distribution.json.

The reference ships no expected outputs for them, so they are configuration fixtures: the tests run
the drop-in workflow with each one on synthetic surfaces and compare with the oracle.  Only the
parsed key = value pairs and the table numbers are stored (data, not the files' text).
Run in the build container only (reads /root/reference):  python tests/golden/make_modified_distribution.py
"""
import json
import os
import sys

SRC = "/root/reference/tests/modified_distribution"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "modified_distribution.json")


def parse_params(path):
    """ParameterReader semantics (ParameterReader.cpp:28-98): 'key = value # comment', keys lower-cased."""
    out = {}
    for line in open(path, encoding="latin-1"):
        line = line.split("#", 1)[0].strip()
        if "=" not in line:
            continue
        k, v = (t.strip() for t in line.split("=", 1))
        if k and v:
            out[k.lower()] = float(v)
    return out


def parse_table(path):
    rows = []
    for line in open(path):
        t = line.split()
        if t:
            rows.append([float(x) for x in t])
    return rows


def main():
    if not os.path.isdir(SRC):
        sys.exit("reference tests/modified_distribution not found")
    cases = {}
    for geom in ("central", "noncentral"):
        for bulk in ("small_bulk", "large_bulk"):
            for df in ("grad", "ce", "ptm", "ptb"):
                for visc in ("none", "shear", "bulk", "shear_bulk"):
                    p = os.path.join(SRC, geom, bulk, "parameters", df, visc, "iS3D_parameters.dat")
                    cases["%s/%s/%s/%s" % (geom, bulk, df, visc)] = parse_params(p)
    tables = {}
    for geom in ("central", "noncentral"):
        tables[geom] = {name: parse_table(os.path.join(SRC, geom, "tables", "%s_table.dat" % name))
                        for name in ("pT", "phi", "y", "eta")}
    chosen = [int(float(t)) for t in open(os.path.join(SRC, "chosen_particles.dat")).read().split()]
    json.dump({"source": "xyw2016/iS3D2 tests/modified_distribution", "chosen": chosen, "tables": tables,
               "cases": cases}, open(OUT, "w"), indent=0, sort_keys=True)
    print("%d cases, chosen %s -> %s" % (len(cases), chosen, OUT))


if __name__ == "__main__":
    main()
