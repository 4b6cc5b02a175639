"""ctypes binding of libpomfret_amd.so (the product: HIP kernels + C ABI).

The library is built in-tree (pomfret_amd/libpomfret_amd.so, see
__graft_entry__.build()).  There is no CPU fallback: if the library or a GPU
is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref

import numpy as np

from .abi import (AlnBatch, Config, KnownVars, LoadConfig, PfAlnBatch, PfCfg, PfKnownVars, PfLoadCfg,
                  PfReadAlnBatch, PfWindowBatch, PfWindowOut, ReadAlnBatch, WindowBatch, WindowResult)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpomfret_amd.so")
_lib = None


class PomfretError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PomfretError(f"{LIB_PATH} not built: run __graft_entry__.build() or "
                               f"`make -C pomfret_amd/csrc`")
        L = C.CDLL(LIB_PATH)
        L.pf_abi_version.restype = C.c_int
        L.pf_device_count.restype = C.c_int
        L.pf_strerror.restype = C.c_char_p
        L.pf_strerror.argtypes = [C.c_int]
        L.pf_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.pf_ctx_destroy.argtypes = [C.c_void_p]
        L.pf_selftest.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.pf_batch_upload.argtypes = [C.c_void_p, C.POINTER(PfCfg), C.POINTER(PfWindowBatch),
                                      C.POINTER(C.c_void_p)]
        L.pf_batch_free.argtypes = [C.c_void_p]
        L.pf_batch_n_windows.argtypes = [C.c_void_p]
        L.pf_batch_n_windows.restype = C.c_uint32
        L.pf_batch_n_reads.argtypes = [C.c_void_p]
        L.pf_batch_n_reads.restype = C.c_uint32
        L.pf_batch_n_calls.argtypes = [C.c_void_p]
        L.pf_batch_n_calls.restype = C.c_uint64
        L.pf_methphase_run.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(PfWindowOut)]
        L.pf_methphase_launch.argtypes = [C.c_void_p, C.c_void_p]
        L.pf_methphase_finish.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(PfWindowOut)]
        L.pf_methphase_windows.argtypes = [C.c_int, C.POINTER(PfCfg), C.POINTER(PfWindowBatch),
                                           C.POINTER(PfWindowOut)]
        L.pf_last_kernel_times.argtypes = [C.c_void_p, C.POINTER(C.c_char_p),
                                           C.POINTER(C.c_float), C.POINTER(C.c_int)]
        L.pf_batch_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.pf_batch_heavy.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32]
        L.pf_batch_k3_paths.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.pf_batch_k12_paths.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.pf_batch_k3_budget.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.pf_batch_debug_sites.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_uint32]
        L.pf_batch_debug_methmers.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                              C.c_void_p, C.c_uint64]
        L.pf_batch_debug_methmers.restype = C.c_int64
        L.pf_fisher_exact.argtypes = [C.c_int] * 4 + [C.POINTER(C.c_double)] * 3
        L.pf_fisher_exact.restype = C.c_double
        L.pf_batch_upload_aln.argtypes = [C.c_void_p, C.POINTER(PfCfg), C.POINTER(PfLoadCfg),
                                          C.POINTER(PfAlnBatch), C.POINTER(C.c_void_p)]
        L.pf_batch_read_recs.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32]
        L.pf_batch_debug_calls.argtypes = [C.c_void_p] + [C.c_void_p] * 5 + [C.c_uint64]
        L.pf_batch_debug_calls.restype = C.c_int64
        L.pf_batch_load_counters.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.pf_batch_debug_recs.argtypes = [C.c_void_p] * 16
        L.pf_bgzf_inflate.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                      C.POINTER(C.c_uint64), C.c_void_p, C.c_uint32, C.POINTER(C.c_float)]
        if hasattr(L, "pf_haptag_reads"):
            L.pf_haptag_reads.argtypes = [C.c_void_p, C.POINTER(PfKnownVars),
                                          C.POINTER(PfReadAlnBatch), C.c_void_p]
        _lib = L
    return _lib


def _check(rc: int, what: str):
    if rc != 0:
        raise PomfretError(f"{what}: {lib().pf_strerror(rc).decode()} ({rc})")


class _PfGaps(C.Structure):
    _fields_ = [("n_contigs", C.c_uint32), ("names", C.POINTER(C.c_char_p)),
                ("abs_start", C.POINTER(C.c_uint32)), ("abs_end", C.POINTER(C.c_uint32)),
                ("raw_off", C.POINTER(C.c_uint64)), ("gap_off", C.POINTER(C.c_uint64)),
                ("drop_off", C.POINTER(C.c_uint64)),
                ("raw_start", C.POINTER(C.c_uint32)), ("raw_end", C.POINTER(C.c_uint32)),
                ("gap_start", C.POINTER(C.c_uint32)), ("gap_end", C.POINTER(C.c_uint32)),
                ("drop_start", C.POINTER(C.c_uint32)), ("drop_end", C.POINTER(C.c_uint32))]


def _gaps_lib():
    L = lib()
    if not getattr(L, "_pf_gaps_typed", False):
        L.pf_vcf_gaps.argtypes = [C.c_char_p, C.c_int32, C.POINTER(C.POINTER(_PfGaps))]
        L.pf_interval_gaps.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.POINTER(C.POINTER(_PfGaps))]
        L.pf_gaps_free.argtypes = [C.POINTER(_PfGaps)]
        L.pf_phase_blocks.argtypes = [C.POINTER(_PfGaps), C.c_void_p, C.POINTER(C.POINTER(_PfBlocks))]
        L.pf_blocks_free.argtypes = [C.POINTER(_PfBlocks)]
        L.pf_write_gtf.argtypes = [C.POINTER(_PfGaps), C.POINTER(_PfBlocks), C.c_char_p]
        L.pf_write_tsv.argtypes = [C.POINTER(_PfGaps), C.POINTER(_PfBlocks), C.c_char_p]
        L.pf_write_vcf.argtypes = [C.c_char_p, C.POINTER(_PfGaps), C.POINTER(_PfBlocks), C.c_void_p,
                                   C.c_char_p, C.POINTER(C.c_int64)]
        L._pf_gaps_typed = True
    return L


class _PfBlocks(C.Structure):
    _fields_ = [("n_contigs", C.c_uint32),
                ("raw_off", C.POINTER(C.c_uint64)), ("dec_off", C.POINTER(C.c_uint64)),
                ("blk_off", C.POINTER(C.c_uint64)),
                ("raw_start", C.POINTER(C.c_uint32)), ("raw_end", C.POINTER(C.c_uint32)),
                ("dec_onraw", C.POINTER(C.c_int32)), ("flip", C.POINTER(C.c_int32)),
                ("blk_start", C.POINTER(C.c_uint32)), ("blk_end", C.POINTER(C.c_uint32))]


def _gaps_contigs(p):
    """pf_gaps_t* -> [dict(name, abs_start, abs_end, raw, gaps, dropped)]."""
    g = p.contents
    res = []
    for c in range(g.n_contigs):
        def sl(off, a, b):
            return [(int(a[k]), int(b[k])) for k in range(off[c], off[c + 1])]
        res.append(dict(name=g.names[c].decode(), abs_start=int(g.abs_start[c]), abs_end=int(g.abs_end[c]),
                        raw=sl(g.raw_off, g.raw_start, g.raw_end), gaps=sl(g.gap_off, g.gap_start, g.gap_end),
                        dropped=sl(g.drop_off, g.drop_start, g.drop_end)))
    return res


def _blocks_contigs(p):
    """pf_blocks_t* -> [dict(raw, decisions, flips, blocks)] per contig."""
    b = p.contents
    res = []
    for c in range(b.n_contigs):
        res.append(dict(
            raw=[(int(b.raw_start[k]), int(b.raw_end[k])) for k in range(b.raw_off[c], b.raw_off[c + 1])],
            decisions=[int(b.dec_onraw[k]) for k in range(b.dec_off[c], b.dec_off[c + 1])],
            flips=[int(b.flip[k]) for k in range(b.dec_off[c], b.dec_off[c + 1])],
            blocks=[(int(b.blk_start[k]), int(b.blk_end[k])) for k in range(b.blk_off[c], b.blk_off[c + 1])]))
    return res


class _PfRescue(C.Structure):
    _fields_ = [("off", C.c_void_p), ("pos", C.c_void_p), ("hap_of_ref", C.c_void_p)]


INTERVALS_VCF, INTERVALS_GTF, INTERVALS_TSV = 0, 1, 2


class Gaps:
    """Phase-block gaps of a phased VCF (pf_vcf_gaps), or of a GTF / 3-column
    TSV of phase blocks (pf_interval_gaps, fmt INTERVALS_GTF / _TSV), owned C
    object."""

    def __init__(self, path: str, readback: int = 50_000, fmt: int = INTERVALS_VCF):
        L = _gaps_lib()
        self._p = C.POINTER(_PfGaps)()
        _check(L.pf_interval_gaps(path.encode(), int(fmt), readback, C.byref(self._p)), "pf_interval_gaps")

    def contigs(self):
        return _gaps_contigs(self._p)

    @property
    def n_windows(self) -> int:
        g = self._p.contents
        return int(g.gap_off[g.n_contigs])

    def close(self):
        if self._p:
            _gaps_lib().pf_gaps_free(self._p)
            self._p = C.POINTER(_PfGaps)()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Blocks:
    """New phase blocks from the join decisions (pf_phase_blocks)."""

    def __init__(self, gaps: Gaps, decision):
        L = _gaps_lib()
        self.gaps = gaps
        self._dec = np.ascontiguousarray(np.asarray(decision, np.int8))
        if self._dec.size != gaps.n_windows:
            raise PomfretError(f"pf_phase_blocks: {self._dec.size} decisions for {gaps.n_windows} windows")
        self._p = C.POINTER(_PfBlocks)()
        _check(L.pf_phase_blocks(gaps._p, self._dec.ctypes.data, C.byref(self._p)), "pf_phase_blocks")

    def contigs(self):
        return _blocks_contigs(self._p)

    def write_gtf(self, path: str):
        _check(_gaps_lib().pf_write_gtf(self.gaps._p, self._p, path.encode()), "pf_write_gtf")

    def write_tsv(self, path: str):
        _check(_gaps_lib().pf_write_tsv(self.gaps._p, self._p, path.encode()), "pf_write_tsv")

    def write_vcf(self, vcf_in: str, vcf_out: str, rescue=None):
        """rescue: optional per-contig list of {pos0: hap_of_ref} dicts."""
        L = _gaps_lib()
        rp = None
        keep = []
        if rescue is not None:
            off = np.zeros(len(rescue) + 1, np.uint64)
            pos, hap = [], []
            for c, m in enumerate(rescue):
                for k in sorted(m):
                    pos.append(k)
                    hap.append(m[k])
                off[c + 1] = len(pos)
            pa = np.asarray(pos, np.uint32) if pos else np.zeros(1, np.uint32)
            ha = np.asarray(hap, np.uint8) if hap else np.zeros(1, np.uint8)
            keep = [off, pa, ha]
            rp = C.byref(_PfRescue(off.ctypes.data, pa.ctypes.data, ha.ctypes.data))
        counts = (C.c_int64 * 3)()
        _check(L.pf_write_vcf(vcf_in.encode(), self.gaps._p, self._p, rp, vcf_out.encode(), counts), "pf_write_vcf")
        del keep
        return tuple(int(x) for x in counts)

    def close(self):
        if self._p:
            _gaps_lib().pf_blocks_free(self._p)
            self._p = C.POINTER(_PfBlocks)()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def vcf_gaps(path: str, readback: int = 50_000):
    """Phase-block gaps of a phased VCF per contig (pf_vcf_gaps): a list of
    dict(name, abs_start, abs_end, raw, gaps, dropped) with (start, end) pairs."""
    return interval_gaps(path, INTERVALS_VCF, readback)


def interval_gaps(path: str, fmt: int = INTERVALS_VCF, readback: int = 50_000):
    """The gaps of any phase-block file `methphase` takes (pf_interval_gaps):
    --vcf, --gtf or --tsv (blockjoin.c:1977-2176, 1305-1345)."""
    g = Gaps(path, readback, fmt)
    res = g.contigs()
    g.close()
    return res


def report_windows(abs_start: int, gaps, chunk_size: int, chunk_stride: int):
    """`pomfret report` chunk windows of one contig (pf_report_windows) from
    its raw gaps [(start, end), ...]."""
    L = lib()
    L.pf_report_windows.restype = C.c_int64
    L.pf_report_windows.argtypes = [C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                    C.c_void_p, C.c_void_p, C.c_uint64]
    gs = np.array([g[0] for g in gaps], np.uint32)
    ge = np.array([g[1] for g in gaps], np.uint32)
    n = L.pf_report_windows(abs_start, gs.ctypes.data, ge.ctypes.data, len(gaps), chunk_size, chunk_stride,
                            None, None, 0)
    _check(0 if n >= 0 else int(n), "pf_report_windows")
    ws = np.zeros(max(n, 1), np.uint32)
    we = np.zeros(max(n, 1), np.uint32)
    L.pf_report_windows(abs_start, gs.ctypes.data, ge.ctypes.data, len(gaps), chunk_size, chunk_stride,
                        ws.ctypes.data, we.ctypes.data, n)
    return list(zip(ws[:n].tolist(), we[:n].tolist()))


def device_count() -> int:
    return int(lib().pf_device_count())


def fisher_exact(n11, n12, n21, n22):
    l, r, t = C.c_double(), C.c_double(), C.c_double()
    q = lib().pf_fisher_exact(n11, n12, n21, n22, C.byref(l), C.byref(r), C.byref(t))
    return q, l.value, r.value, t.value


class Context:
    """One device + one HIP stream (one process per GPU)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        _check(lib().pf_ctx_create(int(device), C.byref(h)), "pf_ctx_create")
        self.handle = h
        self.device = device
        self._batches = weakref.WeakSet()

    def close(self):
        for b in list(self._batches):      # a batch must not outlive its context
            b.free()
        if self.handle:
            lib().pf_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, cfg: Config, batch: WindowBatch) -> "DeviceBatch":
        return DeviceBatch(self, cfg, batch)

    def upload_aln(self, cfg: Config, aln: AlnBatch, lcfg: LoadConfig = None) -> "DeviceBatch":
        """Record-level batch (pf_batch_upload_aln): K0 loads the reads on
        the device in every run."""
        return DeviceBatch(self, cfg, aln, lcfg=lcfg or LoadConfig())

    def bgzf_inflate(self, comp: bytes, out_cap: int = None):
        """Inflate every BGZF block of `comp` on the device (pf_bgzf_inflate).
        Returns (output bytes, per-block status array, inflate kernel ms);
        raises PomfretError when any block fails."""
        comp = np.frombuffer(bytes(comp), np.uint8)
        cap = out_cap if out_cap is not None else max(1, 65536 * (comp.size // 28 + 1))
        out = np.empty(cap, np.uint8)
        n = C.c_uint64()
        st = np.zeros(comp.size // 26 + 1, np.uint32)
        ms = C.c_float()
        rc = lib().pf_bgzf_inflate(self.handle, comp.ctypes.data, comp.size, out.ctypes.data, cap, C.byref(n),
                                   st.ctypes.data, st.size, C.byref(ms))
        self.last_inflate_status = st
        _check(rc, "pf_bgzf_inflate")
        return out[:n.value].tobytes(), st, ms.value

    def kernel_times(self):
        cap = 16
        names = (C.c_char_p * cap)()
        ms = (C.c_float * cap)()
        n = C.c_int(cap)
        _check(lib().pf_last_kernel_times(self.handle, names, ms, C.byref(n)), "kernel_times")
        return {names[i].decode(): float(ms[i]) for i in range(min(n.value, cap))}

    def selftest(self) -> int:
        """Mismatching (a, b) pairs of the kernels' 16-bit count division
        against correctly rounded fp32 division (pf_selftest); 0 expected."""
        n = C.c_uint64(0)
        _check(lib().pf_selftest(self.handle, C.byref(n)), "pf_selftest")
        return int(n.value)

    def haptag_reads(self, known: KnownVars, reads: ReadAlnBatch) -> np.ndarray:
        out = np.zeros(max(reads.n_reads, 1), np.uint8)
        k, r = known.to_c(), reads.to_c()
        _check(lib().pf_haptag_reads(self.handle, C.byref(k), C.byref(r), out.ctypes.data),
               "pf_haptag_reads")
        return out[:reads.n_reads]


class DeviceBatch:
    """A window batch resident in HBM (pf_dbatch_t)."""

    def __init__(self, ctx: Context, cfg: Config, batch, lcfg: LoadConfig = None):
        self.ctx = ctx
        self.n_windows = batch.n_windows
        c, b = cfg.to_c(), batch.to_c()
        h = C.c_void_p()
        if isinstance(batch, AlnBatch):
            lc = lcfg.to_c()
            _check(lib().pf_batch_upload_aln(ctx.handle, C.byref(c), C.byref(lc), C.byref(b), C.byref(h)),
                   "pf_batch_upload_aln")
        else:
            _check(lib().pf_batch_upload(ctx.handle, C.byref(c), C.byref(b), C.byref(h)),
                   "pf_batch_upload")
        self.handle = h
        self.record_level = isinstance(batch, AlnBatch)
        ctx._batches.add(self)

    @classmethod
    def _wrap(cls, ctx: Context, handle, n_windows: int) -> "DeviceBatch":
        """A record-level batch built by the library (e.g. the device fetch)."""
        self = cls.__new__(cls)
        self.ctx = ctx
        self.n_windows = n_windows
        self.handle = handle
        self.record_level = True
        ctx._batches.add(self)
        return self

    def debug_recs(self) -> dict:
        """The record arrays of a record-level batch (pf_batch_debug_recs)."""
        sz = np.zeros(5, np.uint64)
        _check(lib().pf_batch_debug_recs(self.handle, sz.ctypes.data, *([None] * 14)), "pf_batch_debug_recs")
        n, nc, ns, nm, nl = (int(x) for x in sz)
        d = dict(flag=np.zeros(n, np.uint16), mapq=np.zeros(n, np.uint8), pos=np.zeros(n, np.uint32),
                 l_qseq=np.zeros(n, np.uint32), de=np.zeros(n, np.float32), hp=np.zeros(n, np.uint8),
                 cigar_off=np.zeros(n + 1, np.uint64), cigar=np.zeros(max(nc, 1), np.uint32),
                 seq_off=np.zeros(n + 1, np.uint64), seq=np.zeros(max(ns, 1), np.uint8),
                 mm_off=np.zeros(n + 1, np.uint64), mm=np.zeros(max(nm, 1), np.uint8),
                 ml_off=np.zeros(n + 1, np.uint64), ml=np.zeros(max(nl, 1), np.uint8))
        keys = ["flag", "mapq", "pos", "l_qseq", "de", "hp", "cigar_off", "cigar", "seq_off", "seq", "mm_off", "mm",
                "ml_off", "ml"]
        _check(lib().pf_batch_debug_recs(self.handle, sz.ctypes.data, *[d[k].ctypes.data for k in keys]),
               "pf_batch_debug_recs")
        d["cigar"], d["seq"], d["mm"], d["ml"] = d["cigar"][:nc], d["seq"][:ns], d["mm"][:nm], d["ml"][:nl]
        return d

    @property
    def n_reads(self) -> int:
        """Reads of the batch.  Record level: the kept records of the last
        finished run (K0 sizes the batch on the device in every run); before
        any run, the record count (an upper bound)."""
        return int(lib().pf_batch_n_reads(self.handle))

    def read_recs(self) -> np.ndarray:
        """Record index of every read of the batch (identity for window
        batches).  Record level: runs the loader first if no run has finished."""
        R = self.n_reads
        out = np.zeros(max(R, 1), np.uint32)
        rc = lib().pf_batch_read_recs(self.handle, out.ctypes.data, out.size)
        if rc != 0 and self.record_level:           # no run has finished yet: load once
            self.debug_calls(cap=0, probe=True)
            R = self.n_reads
            rc = lib().pf_batch_read_recs(self.handle, out.ctypes.data, out.size)
        _check(rc, "pf_batch_read_recs")
        return out[:R]

    def debug_calls(self, cap: int = None, probe: bool = False):
        """K0 output: (call_off, pos, cat, first, last), calls sorted by (pos, cat) per read.
        probe=True only runs the loader (sizes the batch)."""
        if cap is None:
            if self.record_level and not lib().pf_batch_n_calls(self.handle):
                self.debug_calls(cap=0, probe=True)
            cap = int(lib().pf_batch_n_calls(self.handle))
        R = self.n_reads
        off = np.zeros(R + 1, np.uint64)
        pos = np.zeros(max(cap, 1), np.uint32)
        cat = np.zeros(max(cap, 1), np.uint8)
        first = np.zeros(max(R, 1), np.uint32)
        last = np.zeros(max(R, 1), np.uint32)
        n = lib().pf_batch_debug_calls(self.handle, off.ctypes.data, pos.ctypes.data, cat.ctypes.data,
                                       first.ctypes.data, last.ctypes.data, cap)
        if probe:
            return None
        if n < 0:
            _check(int(n), "pf_batch_debug_calls")
        R = self.n_reads
        return off[:R + 1], pos[:n], cat[:n], first[:R], last[:R]

    def load_counters(self) -> dict:
        out = np.zeros(8, np.uint64)
        _check(lib().pf_batch_load_counters(self.handle, out.ctypes.data, 8), "pf_batch_load_counters")
        return dict(seq_path=int(out[0]), unsorted=int(out[1]), implicit=int(out[2]), bad_mm=int(out[3]),
                    dup_chunks=int(out[4]), multi_cm=int(out[5]))

    def free(self):
        if self.handle:
            lib().pf_batch_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def run(self, out: WindowResult = None) -> WindowResult:
        fresh = out is None
        if fresh:
            out = WindowResult.alloc(self.n_windows, self.n_reads)
        o = out.to_c()
        _check(lib().pf_methphase_run(self.ctx.handle, self.handle, C.byref(o)), "pf_methphase_run")
        if fresh:
            out.read_hp = out.read_hp[:self.n_reads]
        return out

    def stats(self) -> np.ndarray:
        """Per-(window, dir) counters of the last run: [W, 2, 8] (see pf_batch_stats)."""
        out = np.zeros((max(self.n_windows, 1), 2, 8), np.uint64)
        _check(lib().pf_batch_stats(self.handle, out.ctypes.data, out.size), "pf_batch_stats")
        return out[:self.n_windows]

    def k12_paths(self) -> np.ndarray:
        """Per-window sites path of the last run's K12: 1 / 2 the fast path
        over one / two segments, 3 the dense path, 0 none (pf_batch_k12_paths)."""
        out = np.zeros(max(self.n_windows, 1), np.uint8)
        _check(lib().pf_batch_k12_paths(self.handle, out.ctypes.data, out.size), "pf_batch_k12_paths")
        return out[:self.n_windows]

    def k3_paths(self) -> np.ndarray:
        """Per-(window, dir) slot-list source of the last run's greedy loop:
        [W, 2] of 1 LDS lists, 2 candidate cache, 3 HBM lists, 4 general
        body, 5 one-wave kernel, 6 candidate cache with the count table in
        HBM, 0 no sites (pf_batch_k3_paths)."""
        out = np.zeros(max(2 * self.n_windows, 2), np.uint8)
        _check(lib().pf_batch_k3_paths(self.handle, out.ctypes.data, out.size), "pf_batch_k3_paths")
        return out[:2 * self.n_windows].reshape(-1, 2)

    def k3_budget(self) -> dict:
        """The greedy launch of this batch (pf_batch_k3_budget): the main
        kernel's dynamic LDS per problem and its resident workgroups, the
        heavy kernel's LDS and problem count."""
        out = np.zeros(4, np.uint32)
        _check(lib().pf_batch_k3_budget(self.handle, out.ctypes.data, out.size), "pf_batch_k3_budget")
        return {"lds": int(out[0]), "resident": int(out[1]), "lds_heavy": int(out[2]), "n_heavy": int(out[3])}

    def heavy_problems(self) -> np.ndarray:
        """Greedy problems (w<<1 | dir) run in pf_k3_heavy: the windows with at
        least 2,000 reads (1,100 when the batch's 90th-percentile window has
        <= 400), see pf_batch_heavy."""
        n = lib().pf_batch_heavy(self.handle, None, 0)
        out = np.zeros(max(n, 1), np.uint32)
        if n:
            lib().pf_batch_heavy(self.handle, out.ctypes.data, n)
        return out[:n]

    def debug_sites(self, w: int, direction: int, cap: int = 1 << 22):
        real = np.zeros(cap, np.uint32)
        starts = np.zeros(cap, np.uint32)
        lens = np.zeros(cap, np.uint8)
        n = lib().pf_batch_debug_sites(self.handle, w, direction, real.ctypes.data,
                                       starts.ctypes.data, lens.ctypes.data, cap)
        if n < 0:
            _check(n, "pf_batch_debug_sites")
        return real[:n], starts[:n], lens[:n]

    def debug_methmers(self, direction: int, cap: int = 1 << 26):
        n = np.zeros(max(self.n_reads, 1), np.uint32)
        st = np.zeros(max(self.n_reads, 1), np.uint32)
        keys = np.zeros(cap, np.uint32)
        tot = lib().pf_batch_debug_methmers(self.handle, direction, n.ctypes.data, st.ctypes.data,
                                            keys.ctypes.data, cap)
        if tot < 0:
            _check(int(tot), "pf_batch_debug_methmers")
        return n[:self.n_reads], st[:self.n_reads], keys[:tot]

    def launch(self):
        _check(lib().pf_methphase_launch(self.ctx.handle, self.handle), "pf_methphase_launch")

    def finish(self, out: WindowResult = None) -> WindowResult:
        fresh = out is None
        if fresh:
            out = WindowResult.alloc(self.n_windows, self.n_reads)
        o = out.to_c()
        _check(lib().pf_methphase_finish(self.ctx.handle, self.handle, C.byref(o)),
               "pf_methphase_finish")
        if fresh:
            out.read_hp = out.read_hp[:self.n_reads]
        return out


def methphase_windows(cfg: Config, batch: WindowBatch, device: int = 0) -> WindowResult:
    """One-shot: upload + run + free (pf_methphase_windows)."""
    out = WindowResult.alloc(batch.n_windows, batch.n_reads)
    c, b, o = cfg.to_c(), batch.to_c(), out.to_c()
    _check(lib().pf_methphase_windows(int(device), C.byref(c), C.byref(b), C.byref(o)),
           "pf_methphase_windows")
    return out
