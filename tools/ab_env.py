"""A/B of environment knobs on the bench's 1024-window mix batch (seed 1000,
60x, record level) and on its critical window alone: per configuration the
kernel times (mean of `runs` runs, HIP events) and whether the results equal
the first configuration's bit for bit.

usage: python tools/ab_env.py 'NAME:VAR=val,VAR=val' ['NAME2:...' ...]
       (an empty spec 'base:' runs with the environment as is)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import WORKLOAD  # noqa: E402
from pomfret_amd import Config, Context, LoadConfig  # noqa: E402
from pomfret_amd.synth_aln import AlnSpec, load_aln, make_aln_batch, save_aln  # noqa: E402

runs = int(os.environ.get("AB_RUNS", "5"))
nw = int(os.environ.get("AB_WINDOWS", "1024"))
wl = WORKLOAD
cache = os.environ.get("AB_CACHE")           # a .npz: generated once, loaded by later runs
if cache and os.path.exists(cache):
    aln = load_aln(cache)
else:
    aln = make_aln_batch(AlnSpec(n_windows=nw, coverage=60, seed=1000, gap=wl["gap"], gap_mix=wl["gap_mix"],
                                 skip_frac=wl["skip_frac"], nosite_frac=wl["nosite_frac"]), workers=16)
    if cache:
        save_aln(cache, aln)
cfg, lcfg = Config.from_coverage(60, given=False), LoadConfig()
ctx = Context(0)
ref = None
FIELDS = ("decision", "dir_table", "dir_join", "win_n_sites", "win_n_reads", "read_hp", "dir_score")
for spec in sys.argv[1:]:
    name, _, kv = spec.partition(":")
    saved = {}
    for item in filter(None, kv.split(",")):
        k, _, v = item.partition("=")
        saved[k] = os.environ.get(k)
        os.environ[k] = v
    res = {}
    for label, sub in (("batch", aln), ("critical", None)):
        a = sub if sub is not None else aln.select([int(np.argmax(ref_nreads))]) if ref is not None else None
        if a is None:
            continue
        db = ctx.upload_aln(cfg, a, lcfg)
        out = db.run()
        acc = {}
        t0 = time.perf_counter()
        for _ in range(runs):
            db.run()
            for k, v in ctx.kernel_times().items():
                acc[k] = acc.get(k, 0.0) + v / runs
        wall = (time.perf_counter() - t0) / runs * 1e3
        if label == "batch":
            if ref is None:
                ref = out
                ref_nreads = out.win_n_reads
            same = all(np.array_equal(getattr(out, f), getattr(ref, f)) for f in FIELDS)
        else:
            same = None
        import hashlib
        dig = hashlib.sha1(b"".join(np.ascontiguousarray(getattr(out, f)).tobytes() for f in FIELDS)).hexdigest()[:12]
        res[label] = dict(wall_ms=round(wall, 3), same=same, digest=dig, **{k: round(v, 4) for k, v in acc.items() if v > 0.01})
        db.free()
    print(name, res, flush=True)
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
ctx.close()
