"""CPU oracle for Pomfret's methylation-phasing hot path -- TEST INFRASTRUCTURE.

ctypes wrapper around oracle/build/libpf_oracle.so (plain-C restatement of the
reference, oracle/pf_oracle.c).  Only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may import this package; the product
(pomfret_amd/) never does.

Parity status: window definition pinned by the reference's example fixtures;
methylation core "parity unpinned" (reference unbuildable here: htslib absent).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import tempfile

import numpy as np

from pomfret_amd.abi import (AlnBatch, Config, KnownVars, LoadConfig, ReadAlnBatch, WindowBatch,
                             WindowResult)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libpf_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        L.orc_methphase_windows.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_methphase_windows.restype = C.c_int
        L.orc_methphase_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                          C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_window_sites.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int,
                                       C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_window_methmers.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int,
                                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_long]
        L.orc_window_methmers.restype = C.c_long
        L.orc_fisher_exact.argtypes = [C.c_int] * 4 + [C.POINTER(C.c_double)] * 3
        L.orc_fisher_exact.restype = C.c_double
        L.orc_search_arr.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.c_int]
        L.orc_haptag_reads.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_vcf_gaps.argtypes = [C.c_char_p, C.c_int, C.c_char_p]
        L.orc_interval_gaps.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_char_p]
        L.orc_load_reads.argtypes = [C.c_void_p, C.c_void_p] + [C.c_void_p] * 8 + [C.c_uint64, C.c_void_p]
        L.orc_load_reads.restype = C.c_int
        L.orc_methphase_aln.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_methphase_aln.restype = C.c_int
        _lib = L
    return _lib


def methphase(cfg: Config, batch: WindowBatch, n_threads: int = 1) -> WindowResult:
    res = WindowResult.alloc(batch.n_windows, batch.n_reads)
    c, b, o = cfg.to_c(), batch.to_c(), res.to_c()
    rc = lib().orc_methphase_windows(C.byref(c), C.byref(b), C.byref(o), int(n_threads))
    if rc != 0:
        raise RuntimeError(f"oracle failed: {rc}")
    return res


def trace(cfg: Config, batch: WindowBatch, cap: int = 4096):
    W = batch.n_windows
    ids = np.zeros((W, 2, cap), np.uint32)
    tags = np.zeros((W, 2, cap), np.uint8)
    scores = np.zeros((W, 2, cap), np.float32)
    counts = np.zeros((W, 2), np.uint32)
    c, b = cfg.to_c(), batch.to_c()
    lib().orc_methphase_trace(C.byref(c), C.byref(b), cap, ids.ctypes.data, tags.ctypes.data,
                              scores.ctypes.data, counts.ctypes.data)
    return ids, tags, scores, counts


def window_sites(cfg: Config, batch: WindowBatch, w: int, direction: int):
    ro = batch.win_read_off
    co = batch.read_call_off
    cap = int(co[ro[w + 1]] - co[ro[w]]) + 1
    real = np.zeros(cap, np.uint32)
    starts = np.zeros(cap, np.uint32)
    lens = np.zeros(cap, np.uint8)
    c, b = cfg.to_c(), batch.to_c()
    n = lib().orc_window_sites(C.byref(c), C.byref(b), w, direction, real.ctypes.data,
                               starts.ctypes.data, lens.ctypes.data)
    return real[:n], starts[:n], lens[:n]


def window_methmers(cfg: Config, batch: WindowBatch, w: int, direction: int, cap: int = 1 << 22):
    ro = batch.win_read_off
    R = int(ro[w + 1] - ro[w])
    mmr_n = np.zeros(max(R, 1), np.uint32)
    start_i = np.zeros(max(R, 1), np.uint32)
    keys = np.zeros(cap, np.uint32)
    c, b = cfg.to_c(), batch.to_c()
    tot = lib().orc_window_methmers(C.byref(c), C.byref(b), w, direction, mmr_n.ctypes.data,
                                    start_i.ctypes.data, keys.ctypes.data, cap)
    if tot < 0:
        raise RuntimeError("key buffer too small")
    return mmr_n[:R], start_i[:R], keys[:tot]


def fisher(n11, n12, n21, n22):
    l, r, t = C.c_double(), C.c_double(), C.c_double()
    q = lib().orc_fisher_exact(n11, n12, n21, n22, C.byref(l), C.byref(r), C.byref(t))
    return q, l.value, r.value, t.value


def search_arr(a, v, which_end=0):
    a = np.ascontiguousarray(a, np.uint32)
    idx = C.c_uint32(0)
    st = lib().orc_search_arr(a.ctypes.data if len(a) else None, len(a), int(v), C.byref(idx), which_end)
    return st, idx.value


def haptag_reads(known: KnownVars, reads: ReadAlnBatch) -> np.ndarray:
    out = np.zeros(max(reads.n_reads, 1), np.uint8)
    k, r = known.to_c(), reads.to_c()
    lib().orc_haptag_reads(C.byref(k), C.byref(r), out.ctypes.data)
    return out[:reads.n_reads]


def vcf_gaps(path: str, readback: int = 50_000):
    return interval_gaps(path, 0, readback)


INTERVALS_VCF, INTERVALS_GTF, INTERVALS_TSV = 0, 1, 2


def interval_gaps(path: str, fmt: int = INTERVALS_VCF, readback: int = 50_000):
    """load_intervals_from_file (blockjoin.c:1977-2176) for a VCF (PS
    blocks, insert_vcf_line), a GTF (columns 4/5) or a 3-column TSV
    (insert_gtf_line, :1305-1345), then merge_close_intervals(readback)."""
    with tempfile.NamedTemporaryFile("r", suffix=".txt", delete=True) as tf:
        n = lib().orc_interval_gaps(path.encode(), int(fmt), readback, tf.name.encode())
        if n < 0:
            raise RuntimeError(f"vcf_gaps failed {n}")
        out, cur = [], None
        for line in open(tf.name):
            f = line.rstrip("\n").split("\t")
            if f[0] == "contig":
                cur = dict(name=f[1], abs_start=int(f[2]), abs_end=int(f[3]), raw=[], gaps=[], dropped=[])
                out.append(cur)
            else:
                key = {"raw": "raw", "gap": "gaps", "dropped": "dropped"}[f[0]]
                cur[key].append((int(f[1]), int(f[2])))
        return out


def load_reads(lcfg: LoadConfig, aln: AlnBatch):
    """Window loader (a3/a4): the kept reads of every window as a WindowBatch
    (calls in get_mod_poss_on_ref order) and rec_read[r] (read index or
    0xFFFFFFFF for dropped records)."""
    n = aln.n_recs
    rec_read = np.zeros(max(n, 1), np.uint32)
    wro = np.zeros(aln.n_windows + 1, np.uint32)
    rs, re_ = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.uint32)
    rh = np.zeros(max(n, 1), np.uint8)
    co = np.zeros(n + 1, np.uint64)
    cap = int(aln.ml_off[-1]) + int(aln.mm_off[-1]) + int(aln.l_qseq.sum()) // 2 + 16 if n else 16
    need = C.c_uint64(0)
    lc, a = lcfg.to_c(), aln.to_c()
    while True:
        cp, cc = np.zeros(cap, np.uint32), np.zeros(cap, np.uint8)
        R = lib().orc_load_reads(C.byref(lc), C.byref(a), rec_read.ctypes.data, wro.ctypes.data, rs.ctypes.data,
                                 re_.ctypes.data, rh.ctypes.data, co.ctypes.data, cp.ctypes.data, cc.ctypes.data,
                                 cap, C.byref(need))
        if R == -2:
            cap = int(need.value) + 16
            continue
        if R < 0:
            raise RuntimeError(f"oracle load_reads failed: {R}")
        break
    N = int(co[R])
    b = WindowBatch(win_start=aln.win_start, win_end=aln.win_end, win_read_off=wro,
                    read_start=rs[:R], read_end=re_[:R], read_hp=rh[:R], read_call_off=co[:R + 1],
                    call_pos=cp[:N], call_cat=cc[:N], win_cov_sel=aln.win_cov_sel,
                    win_cov_rt=aln.win_cov_rt, win_n_cand=aln.win_n_cand)
    return b, rec_read[:n]


def methphase_aln(cfg: Config, lcfg: LoadConfig, aln: AlnBatch, n_threads: int = 1) -> WindowResult:
    """Record-level path on the CPU (per window: loader a3/a4, then the
    methphase worker).  read_hp is left unset."""
    res = WindowResult.alloc(aln.n_windows, 0)
    c, lc, a, o = cfg.to_c(), lcfg.to_c(), aln.to_c(), res.to_c()
    o.read_hp = None
    rc = lib().orc_methphase_aln(C.byref(c), C.byref(lc), C.byref(a), C.byref(o), int(n_threads))
    if rc != 0:
        raise RuntimeError(f"oracle methphase_aln failed: {rc}")
    return res
