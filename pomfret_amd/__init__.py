"""pomfret_amd -- MI355X-native implementation of Pomfret's per-window
methylation-phasing hot path (the kt_for worker of `pomfret methphase` /
`pomfret report`, reference blockjoin.c:4340-4426 and 4217-4335).

The compute lives in libpomfret_amd.so (hand-written gfx950 HIP kernels behind
a plain C ABI, include/pomfret_amd.h).  This package is the thin Python host
mirror of that interface:

    cfg = Config.from_coverage(30, given=False)     # mmr_config_t derivation
    res = methphase_windows(cfg, batch)             # haplotag_region_given_bam x W
    res.decision                                    # ranges->decisions.a[i]
"""
from .abi import (AlnBatch, Config, KnownVars, LoadConfig, ReadAlnBatch, WindowBatch, WindowResult,
                  HAPTAG_UNPHASED)
from ._lib import (Context, DeviceBatch, PomfretError, device_count, fisher_exact, lib,
                   methphase_windows)

__all__ = [
    "AlnBatch", "Config", "KnownVars", "LoadConfig", "ReadAlnBatch", "WindowBatch", "WindowResult", "HAPTAG_UNPHASED",
    "Context", "DeviceBatch", "PomfretError", "device_count", "fisher_exact", "lib",
    "methphase_windows",
]
