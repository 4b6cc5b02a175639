"""k > 5 greedy paths: one window batch at k (default 6), run under several
greedy-path settings, each run compared with the oracle; the per-problem
slot-list source of every run.  usage: python tools/kdict_diag2.py [k]"""
import dataclasses
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from pomfret_amd import Config, Context  # noqa: E402
from tests._cases import synth  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 6
cfg = dataclasses.replace(Config.from_coverage(30, given=False), k=k)
b = synth(8, 30, 27)
ref = oracle.methphase(cfg, b, n_threads=8)
ctx = Context(0)
F = ("decision", "dir_table", "dir_join", "win_n_sites", "win_n_reads", "read_hp")
for name, env in (("auto", {}), ("auto2", {}), ("lds73k", {"PF_K3_LDS": "73728"}), ("nocache", {"PF_K3_CACHE": "0"}),
                  ("hbm", {"PF_K3_CACHE": "hbm"}), ("force", {"PF_K3_CACHE": "force"}),
                  ("gcnt", {"PF_K3_GCNT": "force"}), ("fold", {"PF_K3_PATH": "fold"})):
    saved = {kk: os.environ.get(kk) for kk in env}
    os.environ.update(env)
    db = ctx.upload(cfg, b)
    res = []
    for it in range(2):
        out = db.run()
        bad = [f for f in F if not np.array_equal(getattr(ref, f), getattr(out, f))]
        res.append(bad)
    paths = db.k3_paths()
    print(name, "mismatch:", res, "paths:", np.unique(paths, return_counts=True), flush=True)
    if res[0]:
        w = np.flatnonzero(ref.decision != out.decision)
        print("   windows", w.tolist(), "paths", paths[w].tolist(), "tables ref", ref.dir_table[w].tolist()[:2],
              "gpu", out.dir_table[w].tolist()[:2], flush=True)
    db.free()
    for kk, v in saved.items():
        if v is None:
            os.environ.pop(kk, None)
        else:
            os.environ[kk] = v
ctx.close()
