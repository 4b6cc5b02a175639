"""`-k` above 5 (VERDICT r05 "next round" 4): methmers of up to 15 characters.

The reference encodes a methmer at 2 bits per character in a u32
(methmer_to_uint32, blockjoin.c:3186-3194; `char mmr[16]`, 3403) and documents
"k is at most 15" (cli.c:243); `-k` itself is taken as given (cli.c:267).  Its
count store is a per-site linear list of the distinct keys
(insert_mmrs_to_counts 3453-3486, query_counts_of_mmrs 3669-3691).  For k <= 5
the greedy kernels number (site, key) slots from a 4^k-bit mask per site; past
that pf_k3_kdict builds per-site hash tables in HBM scratch and ranks each
site's distinct keys -- the same numbering, which PF_K3_KDICT=1 lets the tests
check against the masks at small k.

Parity: every output against the CPU oracle (which takes any k) at k = 6, 8,
11 and 15, on window batches, on a record-level batch (K0 in front), and
through the CLI drop-in (`pomfret-amd methphase -k 6 / -k 8`).
"""
import dataclasses
import os

import numpy as np
import pytest

from tests import _fixtures as fx
from tests._cases import synth
from tests._oracle_pipeline import methphase_files_oracle
from tests.test_parity_gpu import _compare

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(k, cov=30, **kw):
    from pomfret_amd import Config
    return dataclasses.replace(Config.from_coverage(cov, given=False), k=k, **kw)


@pytest.mark.parametrize("k", [6, 8, 11, 15])
def test_large_k_windows_parity(oracle_lib, gpu_ctx, k):
    """Decisions, tables, joins, site counts, read tags and Fisher p equal the
    oracle's with k-character methmers (a 30x batch and a gap-mix batch)."""
    for name, batch in (("synth30", synth(8, 30, 21 + k)), ("gapmix", synth(6, 30, 60 + k, gap_mix=True))):
        cfg = _cfg(k)
        ref = oracle_lib.methphase(cfg, batch, n_threads=8)
        db = gpu_ctx.upload(cfg, batch)
        out = db.run()
        _compare(ref, out, f"k{k} {name}")
        # every greedy problem with sites ran (no silent empty table)
        assert (out.win_n_sites > 0).sum() >= batch.n_windows // 2
        db.free()


@pytest.mark.parametrize("k", [6, 15])
def test_large_k_methmer_keys(oracle_lib, gpu_ctx, k):
    """The keys themselves (before the dictionary rewrites them): every read's
    methmer list equals get_mmr_of_read's, 2 bits per character."""
    batch = synth(4, 30, 90 + k)
    cfg = _cfg(k)
    db = gpu_ctx.upload(cfg, batch)
    ro = batch.win_read_off
    for d in (0, 1):
        n, st, keys = db.debug_methmers(d)
        k0 = 0
        for w in range(batch.n_windows):
            on, ost, okeys = oracle_lib.window_methmers(cfg, batch, w, d)
            assert np.array_equal(on, n[ro[w]:ro[w + 1]]), f"k{k} w{w} d{d} mmr_n"
            assert np.array_equal(ost, st[ro[w]:ro[w + 1]]), f"k{k} w{w} d{d} mmr_start"
            assert np.array_equal(okeys, keys[k0:k0 + len(okeys)]), f"k{k} w{w} d{d} keys"
            k0 += len(okeys)
        if k == 15:
            assert int(np.max(keys)) >= 1 << 20      # long keys really occur
    db.free()


@pytest.mark.parametrize("k", [1, 3, 5])
def test_hash_dictionary_equals_masks(gpu_ctx, monkeypatch, k):
    """PF_K3_KDICT=1 takes the hash-table dictionary at k <= 5: the slots, and
    so every output, equal the mask dictionary's bit for bit (60x gap mix,
    where windows run through every greedy path)."""
    batch = synth(16, 60, 300 + k, gap_mix=True)
    cfg = _cfg(k, cov=60)
    outs = []
    for kd in ("0", "1"):
        monkeypatch.setenv("PF_K3_KDICT", kd)
        db = gpu_ctx.upload(cfg, batch)
        outs.append(db.run())
        db.free()
    _compare(outs[0], outs[1], f"kdict k{k}")


def test_large_k_record_level(oracle_lib, gpu_ctx):
    """K0 in front: a record-level batch at k = 8 equals the oracle pipeline
    (load_reads_given_interval then the window worker)."""
    from pomfret_amd import LoadConfig
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    aln = make_aln_batch(AlnSpec(n_windows=3, coverage=30, seed=808, len_scale=0.6))
    cfg = _cfg(8)
    db = gpu_ctx.upload_aln(cfg, aln, LoadConfig())
    out = db.run()
    # the oracle's loader, then its window worker (methphase_aln leaves the read tags unset)
    wb = oracle_lib.load_reads(LoadConfig(), aln)[0]
    ref = oracle_lib.methphase(cfg, wb, n_threads=8)
    _compare(ref, out, "aln k8")
    db.free()


@pytest.mark.parametrize("k", [6, 8])
def test_cli_large_k(oracle_lib, tmp_path, k):
    """`pomfret-amd methphase -k K -c 30 --vcf v.vcf t.bam` runs (round 5
    refused k > 5) and writes the oracle pipeline's GTF / TSV / VCF bytes."""
    import subprocess
    from pomfret_amd import Config
    aln, recs, bam, vcf = fx.tagged(tmp_path, n_windows=4)
    out = str(tmp_path / f"k{k}")
    exe = os.path.join(ROOT, "pomfret_amd", "pomfret-amd")
    r = subprocess.run([exe, "methphase", "-k", str(k), "-o", out, "-c", "30", "--vcf", vcf, "--output-tsv", bam],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    cfg = dataclasses.replace(Config.from_coverage(30, given=True), k=k)
    ref = methphase_files_oracle(bam, vcf, cfg, recs_by_contig={"chrS": recs})
    assert (ref["decision"] >= 0).sum() >= 1     # longer methmers join fewer of these 4 windows
    assert open(out + ".mp.gtf").read() == ref["gtf"]
    assert open(out + ".mp.tsv").read() == ref["tsv"]
    assert open(out + ".mp.vcf", "rb").read() == ref["vcf"]


def test_k_above_15_refused(gpu_ctx):
    """k > 15 overflows the reference's u32 encoding and its 16-byte buffer:
    the library refuses it instead of computing something else."""
    from pomfret_amd._lib import PomfretError
    batch = synth(2, 30, 5)
    with pytest.raises(PomfretError, match="unsupported"):
        gpu_ctx.upload(_cfg(16), batch)
