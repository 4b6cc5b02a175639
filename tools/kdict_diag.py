"""Diagnostic for the k > 5 path (pf_k3_kdict): one window batch at the given
k, staged (K12/K2 keys against the oracle, then the whole run against the
oracle).  usage: python tools/kdict_diag.py K [PF_K3_KDICT]"""
import dataclasses
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from pomfret_amd import Config, Context  # noqa: E402
from tests._cases import synth  # noqa: E402

k = int(sys.argv[1])
if len(sys.argv) > 2:
    os.environ["PF_K3_KDICT"] = sys.argv[2]
cfg = dataclasses.replace(Config.from_coverage(30, given=False), k=k)
b = synth(8, 30, 27)
ctx = Context(0)
db = ctx.upload(cfg, b)
ro = b.win_read_off
for d in (0, 1):
    n, st, keys = db.debug_methmers(d)
    k0 = 0
    for w in range(b.n_windows):
        on, ost, okeys = oracle.window_methmers(cfg, b, w, d)
        assert np.array_equal(on, n[ro[w]:ro[w + 1]]), f"w{w} d{d} mmr_n"
        assert np.array_equal(okeys, keys[k0:k0 + len(okeys)]), f"w{w} d{d} keys"
        k0 += len(okeys)
print("methmers ok", flush=True)
out = db.run()
ref = oracle.methphase(cfg, b, n_threads=8)
for f in ("decision", "dir_table", "dir_join", "win_n_sites", "win_n_reads", "read_hp"):
    assert np.array_equal(getattr(ref, f), getattr(out, f)), f
print("run ok", flush=True)
db.free()
ctx.close()
