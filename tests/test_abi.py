"""CPU tests of the C ABI library: it loads, exports every entry point that
include/pomfret_amd.h declares, and its host-side pieces behave (no GPU)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "pomfret_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pf_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from pomfret_amd import lib
    L = lib()
    names = _declared()
    assert "pf_methphase_windows" in names and "pf_haptag_reads" in names
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, f"not exported: {missing}"


def test_abi_version_and_errors():
    from pomfret_amd import lib
    L = lib()
    assert L.pf_abi_version() == 1
    assert L.pf_strerror(-5) == b"input exceeds a documented limit"


def test_struct_layouts_match_header():
    """ctypes mirrors (pomfret_amd/abi.py) have the C layout sizes."""
    from pomfret_amd.abi import PfCfg, PfKnownVars, PfReadAlnBatch, PfWindowBatch, PfWindowOut
    assert C.sizeof(PfCfg) == 32
    assert C.sizeof(PfWindowBatch) == 4 + 4 + 8 + 12 * 8
    assert C.sizeof(PfWindowOut) == 9 * 8
    assert C.sizeof(PfKnownVars) == 8 + 6 * 8
    assert C.sizeof(PfReadAlnBatch) == 8 + 9 * 8


def test_no_device_is_an_error_not_a_fallback():
    """Without a GPU the product refuses to run (no CPU fallback path)."""
    from pomfret_amd import Config, PomfretError, device_count, methphase_windows
    from pomfret_amd.synth import SynthSpec, make_batch
    if device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(PomfretError):
        methphase_windows(Config(), make_batch(SynthSpec(n_windows=1)))


def test_config_derivation():
    """cov_for_selection / cov_for_runtime / n_cand as the reference derives them."""
    from pomfret_amd import Config
    c = Config.from_coverage(60, given=True)      # methphase -c 60 (cli.c:270-275)
    assert (c.cov_for_selection, c.cov_for_runtime, c.n_cand) == (6, 12, 15)
    c = Config.from_coverage(30, given=False)     # auto estimate (blockjoin.c:4373-4375)
    assert (c.cov_for_selection, c.cov_for_runtime, c.n_cand) == (4, 8, 8)
    c = Config.from_coverage(200, report=True)    # report (blockjoin.c:5045-5051)
    assert (c.cov_for_selection, c.cov_for_runtime, c.n_cand) == (21, 42, 51)
    c = Config.from_coverage(4, given=True)       # clamps (blockjoin.c:4381-4390)
    assert (c.cov_for_selection, c.n_cand) == (1, 2)


def test_host_epilogue_decisions():
    """pf_host.c decision logic on hand tables (evaluate_separation1,
    blockjoin.c:3881-3939 + the join rule of :4147-4156)."""
    from pomfret_amd import lib
    L = lib()
    L.pf_evaluate_table.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_double)]
    L.pf_evaluate_table.restype = C.c_float
    L.pf_join_from_eval.argtypes = [C.c_float, C.c_int]

    def ev(t):
        a = np.array(t, np.int32)
        w, p = C.c_int(), C.c_double()
        s = L.pf_evaluate_table(a.ctypes.data, C.byref(w), C.byref(p))
        return s, w.value, p.value, L.pf_join_from_eval(s, w.value)

    s, w, p, j = ev([20, 0, 0, 18])       # cis: raw hap == new hap
    assert (w, j) == (2, 0) and s == 18.0 and p < 1e-3
    s, w, p, j = ev([0, 14, 15, 0])       # trans
    assert (w, j) == (-2, 1)
    assert ev([20, 6, 0, 18])[1] == -9    # contamination > 5 in one row
    assert ev([5, 2, 0, 9])[1] == -9      # ratio 5/2 < 3
    assert ev([3, 0, 0, 3])[3] == -1      # not significant (p >= 0.001)


def test_ingest_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of the host-ingest structs (pomfret_amd/bam.py) against
    the C compiler's sizeof / offsetof of include/pomfret_amd.h."""
    import subprocess
    from pomfret_amd.abi import PfAlnBatch
    from pomfret_amd.bam import PfBamReads, PfBamRecords, PfKnownTable, PfQnameTags, PfRescueMap
    src = tmp_path / "l.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "pomfret_amd.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(pf_aln_batch_t),'
                   'sizeof(pf_bam_records_t), offsetof(pf_bam_records_t, n_truncated), sizeof(pf_bam_reads_t),'
                   'sizeof(pf_known_table_t), sizeof(pf_qname_tags_t), sizeof(pf_rescue_map_t),'
                   'offsetof(pf_bam_reads_t, qname));return 0;}\n')
    exe = tmp_path / "l"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    exp = [C.sizeof(PfAlnBatch), C.sizeof(PfBamRecords), PfBamRecords.n_truncated.offset, C.sizeof(PfBamReads),
           C.sizeof(PfKnownTable), C.sizeof(PfQnameTags), C.sizeof(PfRescueMap), PfBamReads.qname.offset]
    assert got == exp
