"""Output epilogue, CPU only.

The product (pomfret_amd/csrc/pf_epilogue.c: pf_phase_blocks, pf_write_gtf,
pf_write_tsv, pf_write_vcf) is checked
  * against the reference's own example fixture (tests/golden/example): the
    one TRANS join of its single gap rewrites the VCF byte for byte as the
    committed output.mp.vcf, except the variant AT abs_end, which the golden
    output (an older reference build) still re-phases and
    the current reference excludes ([s, e) at blockjoin.c:2377); the GTF
    differs from the golden only by the tab the older build's format string
    lacked after the end column;
  * against the oracle's pure-Python restatement (oracle/epilogue.py) on
    seeded synthetic VCFs: several contigs, merged gaps with dropped
    intervals, random decisions, rescued dropped sites, FORMAT with PS before
    GT, homozygous and multi-allelic phased GTs, PS ".", unphased GTs, a POS
    decrease at a contig switch and none at another.
"""
import os
import random

import pytest

from pomfret_amd import _lib

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "example")
HEADER = "##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\n"


def test_example_fixture(oracle_lib, tmp_path):
    from oracle import epilogue as ep
    vin = os.path.join(GOLD, "variants.vcf.gz")
    g = _lib.Gaps(vin)
    b = _lib.Blocks(g, [1])                       # the golden run joined the gap TRANS
    out = str(tmp_path / "o.vcf")
    counts = b.write_vcf(vin, out)
    got = open(out, "rb").read()
    gold = open(os.path.join(GOLD, "output.mp.vcf"), "rb").read()
    gl, gg = got.split(b"\n"), gold.split(b"\n")
    assert len(gl) == len(gg)
    abs_end = g.contigs()[0]["abs_end"]
    diff = [i for i in range(len(gl)) if gl[i] != gg[i]]
    assert len(diff) == 1
    line = gl[diff[0]].split(b"\t")
    assert int(line[1]) == abs_end                # the [s, e) exclusion of abs_end
    assert counts == (24, 0, 346)
    # GTF: identical up to the missing tab of the older build
    b.write_gtf(str(tmp_path / "o.gtf"))
    gtf = open(tmp_path / "o.gtf").read()
    assert gtf.replace("\t.\t+", ".\t+", 1) == open(os.path.join(GOLD, "output.mp.gtf")).read()
    # the oracle restatement agrees with the product on the fixture
    oc = oracle_lib.vcf_gaps(vin)
    ob = ep.phase_blocks(oc, [1])
    assert ob == b.contigs()
    ov, ocounts = ep.vcf_bytes(vin, oc, ob)
    assert ov == got and ocounts == counts
    assert ep.gtf_text(oc, ob) == gtf


def _synth(rng):
    """Phased VCF with several contigs; blocks separated by gaps of mixed
    sizes (some below the 50 kb readback, so they merge and drop)."""
    lines, truth_pos = [], {}
    n_ctg = rng.randrange(1, 4)
    last = 0
    for ci in range(n_ctg):
        name = f"chr{ci + 1}"
        # sometimes restart POS below the previous contig's last POS (flip
        # cursor reset), sometimes continue above it (no reset)
        pos = rng.randrange(1000, 50_000) if (ci == 0 or rng.random() < 0.5) else last + rng.randrange(10, 1000)
        for _ in range(rng.randrange(1, 9)):
            block0 = pos
            for _ in range(rng.randrange(1, 12)):
                r = rng.random()
                gt = rng.choice(["0|1", "1|0", "0|1", "1|0", "0|0", "1|1", "1|2", "0/1"])
                ps = "." if r < 0.05 else str(block0)
                if r < 0.1:
                    fmt, smp = "GT", "0/1"
                elif r < 0.25:
                    fmt, smp = "PS:GT:GQ", f"{ps}:{gt}:30"
                else:
                    fmt, smp = "GT:GQ:PS", f"{gt}:30:{ps}"
                lines.append(f"{name}\t{pos}\t.\tA\tC\t50\tPASS\t.\t{fmt}\t{smp}\n")
                truth_pos.setdefault(ci, []).append(pos)
                pos += rng.randrange(1, 4000)
            pos += rng.choice([100, 5000, 20_000, 60_000, 150_000])
        last = pos
    return HEADER + "".join(lines), n_ctg, truth_pos


@pytest.mark.parametrize("seed", range(16))
def test_synthetic_matches_oracle(oracle_lib, tmp_path, seed):
    from oracle import epilogue as ep
    rng = random.Random(seed)
    text, n_ctg, truth_pos = _synth(rng)
    vin = str(tmp_path / "v.vcf")
    open(vin, "w").write(text)
    g = _lib.Gaps(vin)
    oc = oracle_lib.vcf_gaps(vin)
    assert g.contigs() == oc
    dec = [rng.choice([-1, 0, 1, 1]) for _ in range(g.n_windows)]
    b = _lib.Blocks(g, dec)
    ob = ep.phase_blocks(oc, dec)
    assert b.contigs() == ob
    # rescue maps: some 0-based positions of variants inside dropped intervals
    rescue = []
    for ci, c in enumerate(oc):
        m = {}
        for p in truth_pos.get(ci, []):
            if any(ds <= p <= de for ds, de in c["dropped"]) and rng.random() < 0.6:
                m[p - 1] = rng.choice([0, 1, 254])
        rescue.append(m)
    for resc in (None, rescue):
        out = str(tmp_path / "o.vcf")
        counts = b.write_vcf(vin, out, resc)
        ov, ocounts = ep.vcf_bytes(vin, oc, ob, resc)
        assert open(out, "rb").read() == ov
        assert counts == ocounts
    b.write_gtf(str(tmp_path / "o.gtf"))
    b.write_tsv(str(tmp_path / "o.tsv"))
    assert open(tmp_path / "o.gtf").read() == ep.gtf_text(oc, ob)
    assert open(tmp_path / "o.tsv").read() == ep.tsv_text(oc, ob)


def test_all_joined_and_none_joined(oracle_lib, tmp_path):
    """All gaps joined: one block per contig from abs_start; none joined:
    blocks between the gaps and the last from the last gap's start."""
    from oracle import epilogue as ep
    rng = random.Random(99)
    text, _, _ = _synth(rng)
    vin = str(tmp_path / "v.vcf")
    open(vin, "w").write(text)
    g = _lib.Gaps(vin)
    oc = oracle_lib.vcf_gaps(vin)
    for d in (0, 1, -1):
        dec = [d] * g.n_windows
        b = _lib.Blocks(g, dec)
        assert b.contigs() == ep.phase_blocks(oc, dec)
        for c, bc in zip(oc, b.contigs()):
            if d >= 0 and c["gaps"]:
                assert bc["blocks"][0][0] == c["abs_start"]


def test_bad_header_and_counts(tmp_path):
    vin = str(tmp_path / "v.vcf")
    open(vin, "w").write(HEADER + "c\t100\t.\tA\tC\t50\tPASS\t.\tGT:PS\t0|1:100\n"
                         "c\t200\t.\tA\tC\t50\tPASS\t.\tGT:PS\t0|1:200\n")
    g = _lib.Gaps(vin)
    b = _lib.Blocks(g, [1])
    bad = str(tmp_path / "bad.vcf")
    open(bad, "w").write("#CHROM\tPOS\n")
    with pytest.raises(_lib.PomfretError):
        b.write_vcf(bad, str(tmp_path / "o.vcf"))
    with pytest.raises(_lib.PomfretError):
        _lib.Blocks(g, [1, 0])                     # wrong number of decisions
