import sys, numpy as np
sys.path[:0]=["/root/repo","/root/repo/tests"]
import torch; torch.cuda.init()
from helpers import parity, rel_quantile
from is3d2_amd import build_engine, make_spec, synth
from oracle import oracle as O
def run(spec, s, tuning=None):
    e = build_engine(spec, s)
    for k, v in (tuning or {}).items(): e.set_tuning(k, v)
    out = e.calculate_spectra(); ch = e.get_tuning("phitab_chunks"); sp=e.get_tuning("splits"); sl=e.get_tuning("slabs"); e.close(); return out, ch, sp, sl
for n in (48, 96):
    s = synth.as_read(synth.surface(n, seed=29, dimension=3, baryon=True, full3d=True))
    hot = np.arange(n) % 2 == 0
    s["T"] = np.where(hot, 0.12, s["T"]); s["muB"] = np.where(hot, 45.0, s["muB"])
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=1, dimension=3, pT="pT24", phi="phi32", y="y21", include_baryon=1)
    T, muB, tab = spec["df"]; spec["df"] = (T, np.asarray(muB) * 100.0, tab)
    ref = O.spectra(spec, s, threads=8)
    for tun in (None, {"phitab_one_bytes": 0, "phitab_chunk_bytes": 1}):
        got, ch, sp, sl = run(spec, s, tun)
        m = np.abs(ref) > 1e-300
        rel = np.abs(got[m]-ref[m])/np.abs(ref[m])
        i = np.argmax(rel)
        print(n, tun is not None, "chunks", ch, "splits", sp, "slabs", sl, "max rel %.3g at ref %.3g got %.3g" % (rel[i], ref[m][i], got[m][i]), "p99 %.3g" % np.quantile(rel, 0.99), "n>1e-8:", int((rel>1e-8).sum()), flush=True)
