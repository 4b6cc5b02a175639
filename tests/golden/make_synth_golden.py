"""Generates tests/golden/synth_oracle.npz: oracle outputs on small seeded
synthetic batches, committed as a regression pin of the oracle (they are NOT
reference outputs: the reference cannot be built here)."""
import dataclasses
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from pomfret_amd.abi import Config  # noqa: E402
from pomfret_amd.synth import SynthSpec, make_batch  # noqa: E402
import oracle  # noqa: E402

CASES = {
    "c30": (SynthSpec(n_windows=6, coverage=30, seed=101), Config.from_coverage(30, given=False)),
    "c60": (SynthSpec(n_windows=4, coverage=60, seed=102), Config.from_coverage(60, given=True)),
    "mix": (SynthSpec(n_windows=5, coverage=30, seed=103, gap_mix=True), Config.from_coverage(30, given=False)),
}

if __name__ == "__main__":
    out = {}
    for tag, (spec, cfg) in CASES.items():
        b = make_batch(spec)
        res = oracle.methphase(cfg, b, n_threads=4)
        d = dataclasses.asdict(spec)
        out[f"{tag}_spec_keys"] = np.array(list(d.keys()))
        out[f"{tag}_spec_vals"] = np.array([int(v) if isinstance(v, (bool, int)) else v for v in d.values()], dtype=object).astype(float)
        out[f"{tag}_cfg"] = np.array(dataclasses.astuple(cfg), np.int64)
        out[f"{tag}_decision"] = res.decision
        out[f"{tag}_table"] = res.dir_table
        out[f"{tag}_sites"] = res.win_n_sites
        out[f"{tag}_hp"] = res.read_hp
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "synth_oracle.npz"), **out)
    print("wrote", {k: v.shape for k, v in out.items() if k.endswith("decision")})
