"""Seeded synthetic long-read methylation pileups.

HG002 data is not available offline, so both the parity tests and the
benchmark run on synthetic windows shaped like the reference's inputs after
its BAM window loader (reference blockjoin.c:1043-1173):

* window = one phasing gap [s, e] of length `gap`; reads are those overlapping
  the fetch region [s - readback, e + readback] (blockjoin.c:1053-1054);
* read length lognormal (mean 30 kb, sd 15 kb) clipped to [15 kb, 150 kb]
  (so every read passes the -L 15000 filter), strand Bernoulli(0.5);
* CpGs Poisson at 1/100 bp; site classes 70 % methylated (p=0.95),
  20 % unmethylated (p=0.05), 10 % allele-specific (0.95/0.05 by haplotype);
* call category per ML qual bands: meth U[200,255] -> 0, unmeth U[0,95] -> 1,
  5 % in the no-call band U[100,155] -> 2 (lo=100, hi=156, blockjoin.c:876-878);
* truth haplotype uniform; reads touching the left block carry HP=truth+1,
  reads touching only the right block carry HP=(truth xor orientation)+1,
  reads inside the gap (and `untag_frac` of the rest) are untagged (254);
  orientation (cis/trans) is drawn per window.

Everything is a pure function of (seed, window index), so any sub-batch of
windows is reproducible on its own.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .abi import HAPTAG_UNPHASED, WindowBatch


@dataclass
class SynthSpec:
    n_windows: int = 256
    coverage: float = 30.0
    gap: int = 50_000
    readback: int = 50_000
    mean_len: float = 30_000.0
    sd_len: float = 15_000.0
    min_len: int = 15_000
    max_len: int = 150_000
    cpg_rate: float = 0.01
    nocall_frac: float = 0.05
    untag_frac: float = 0.10
    seed: int = 1
    window_stride: int = 600_000
    base: int = 1_000_000
    gap_mix: bool = False      # log-uniform 5-500 kb gap lengths instead of fixed


def _lognormal_params(mean: float, sd: float):
    sigma2 = np.log(1.0 + (sd / mean) ** 2)
    return np.log(mean) - sigma2 / 2.0, np.sqrt(sigma2)


def make_window(spec: SynthSpec, w: int):
    """Returns dict with s, e, reads (start,end,hp) and their calls."""
    rng = np.random.default_rng([spec.seed, w])
    gap = spec.gap
    if spec.gap_mix:
        gap = int(np.exp(rng.uniform(np.log(5_000), np.log(500_000))))
    stride = max(spec.window_stride, gap + 2 * spec.readback + 2 * spec.max_len + 10_000)
    # windows are independent: the layout wraps below the 2^29 position limit
    s = spec.base + (w % max(1, (400_000_000 - spec.base) // stride)) * stride
    e = s + gap
    f_lo, f_hi = max(0, s - spec.readback), e + spec.readback
    span_lo, span_hi = f_lo - spec.max_len, f_hi + spec.max_len

    # CpGs
    n_cpg = rng.poisson(spec.cpg_rate * (span_hi - span_lo))
    cpg = np.unique(rng.integers(span_lo, span_hi, size=n_cpg, dtype=np.int64))
    n_cpg = cpg.shape[0]
    cls = rng.random(n_cpg)
    p_meth = np.where(cls < 0.7, 0.95, 0.05)            # [0,0.7) meth, [0.7,0.9) unmeth
    asm = cls >= 0.9                                     # allele specific
    asm_hap = rng.integers(0, 2, n_cpg)

    # reads
    mu, sig = _lognormal_params(spec.mean_len, spec.sd_len)
    n_draw = int(spec.coverage * (span_hi - span_lo) / spec.mean_len)
    starts = rng.integers(span_lo, f_hi, size=n_draw, dtype=np.int64)
    lens = np.clip(np.exp(rng.normal(mu, sig, n_draw)), spec.min_len, spec.max_len).astype(np.int64)
    ends = starts + lens
    keep = (ends > f_lo) & (starts < f_hi) & (starts >= 0)
    starts, ends = starts[keep], ends[keep]
    order = np.argsort(starts, kind="stable")
    starts, ends = starts[order], ends[order]
    n = starts.shape[0]
    truth = rng.integers(0, 2, n)
    orient = int(rng.integers(0, 2))
    hp = np.full(n, HAPTAG_UNPHASED, np.int64)
    touches_left = starts < s
    touches_right = ends > e
    hp[touches_left] = truth[touches_left]
    only_right = (~touches_left) & touches_right
    hp[only_right] = truth[only_right] ^ orient
    untag = rng.random(n) < spec.untag_frac
    hp[untag] = HAPTAG_UNPHASED

    # calls: every CpG inside [start, end)
    lo = np.searchsorted(cpg, starts, side="left")
    hi = np.searchsorted(cpg, ends, side="left")
    cnt = hi - lo
    tot = int(cnt.sum())
    read_of_call = np.repeat(np.arange(n), cnt)
    first = np.repeat(lo - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt)
    idx = np.arange(tot) + first
    p = p_meth[idx].copy()
    a = asm[idx]
    p[a] = np.where(asm_hap[idx][a] == truth[read_of_call][a], 0.95, 0.05)
    is_meth = rng.random(tot) < p
    cat = np.where(is_meth, 0, 1).astype(np.uint8)
    cat[rng.random(tot) < spec.nocall_frac] = 2

    # load_reads_given_interval keeps only reads with >= 1 call (blockjoin.c:933-936)
    has = cnt > 0
    if not has.all():
        keep_call = has[read_of_call]
        idx, cat = idx[keep_call], cat[keep_call]
        starts, ends, hp, cnt = starts[has], ends[has], hp[has], cnt[has]
    return dict(s=s, e=e, orient=orient, read_start=starts, read_end=ends, read_hp=hp,
                call_cnt=cnt, call_pos=cpg[idx], call_cat=cat)


def make_batch(spec: SynthSpec, windows=None) -> WindowBatch:
    if windows is None:
        windows = range(spec.n_windows)
    parts = [make_window(spec, w) for w in windows]
    rc = np.array([p["read_start"].shape[0] for p in parts], np.int64)
    ccnt = np.concatenate([p["call_cnt"] for p in parts]) if parts else np.zeros(0, np.int64)
    b = WindowBatch(
        win_start=np.array([p["s"] for p in parts], np.uint32),
        win_end=np.array([p["e"] for p in parts], np.uint32),
        win_read_off=np.concatenate([[0], np.cumsum(rc)]).astype(np.uint32),
        read_start=np.concatenate([p["read_start"] for p in parts]).astype(np.uint32),
        read_end=np.concatenate([p["read_end"] for p in parts]).astype(np.uint32),
        read_hp=np.concatenate([p["read_hp"] for p in parts]).astype(np.uint8),
        read_call_off=np.concatenate([[0], np.cumsum(ccnt)]).astype(np.uint64),
        call_pos=np.concatenate([p["call_pos"] for p in parts]).astype(np.uint32),
        call_cat=np.concatenate([p["call_cat"] for p in parts]).astype(np.uint8),
    )
    b.meta["orient"] = np.array([p["orient"] for p in parts], np.int8)
    b.meta["spec"] = spec
    return b
