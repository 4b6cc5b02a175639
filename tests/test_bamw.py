"""--write-bam and varhaptag output: pf_retag_bam on the CPU.

The output BAM is parsed by an independent test-side reader and checked
record by record against the input: identical bytes except the HP tag, whose
value follows a Python restatement of output_modify_bam
(blockjoin.c:3022-3103: check_if_in_phased_intervals, get_flip_status_by_idx
and get_read_new_haplotag with their index quirks) or of main_varhaptag
(4737-4836), written as htslib's bam_aux_update_int writes it.  The BGZF
layout follows bgzf_write/bgzf_flush_try (header in its own block, records
never straddling blocks unless larger than one), and the index is checked by
region queries of the library's reader against the overlap rule.  htslib
itself is absent, so byte identity with htslib's output is unpinned."""
import os
import random
import struct
import zlib

import numpy as np
import pytest

from tests._bamio import Rec, aux_C, aux_f, aux_i, aux_Z, endpos, expected_fetch, write_bam, write_phased_vcf

SHORT = {"c": ("<b", 1), "C": ("<B", 1), "s": ("<h", 2), "S": ("<H", 2), "i": ("<i", 4), "I": ("<I", 4)}


def read_bgzf_blocks(path):
    """[(compressed offset, uncompressed bytes)] of every block."""
    raw = open(path, "rb").read()
    out, o = [], 0
    while o < len(raw):
        assert raw[o:o + 4] == b"\x1f\x8b\x08\x04"
        xlen = struct.unpack_from("<H", raw, o + 10)[0]
        bsize = struct.unpack_from("<H", raw, o + 16)[0] + 1
        data = zlib.decompress(raw[o + 12 + xlen:o + bsize - 8], -15)
        assert zlib.crc32(data) == struct.unpack_from("<I", raw, o + bsize - 8)[0]
        out.append((o, data))
        o += bsize
    return out


def parse_bam(path):
    """(header bytes, [record body bytes], [virtual offset of each record], block starts)"""
    blocks = read_bgzf_blocks(path)
    starts, parts, n = [], [], 0
    for off, data in blocks:
        starts.append((off, n))
        parts.append(data)
        n += len(data)
    buf = b"".join(parts)
    lt = struct.unpack_from("<i", buf, 4)[0]
    o = 8 + lt
    nref = struct.unpack_from("<i", buf, o)[0]
    o += 4
    for _ in range(nref):
        ln = struct.unpack_from("<i", buf, o)[0]
        o += 4 + ln + 4
    hdr_end = o
    recs, voffs = [], []
    while o < len(buf):
        bs = struct.unpack_from("<i", buf, o)[0]
        voffs.append(o)
        recs.append(buf[o + 4:o + 4 + bs])
        o += 4 + bs
    return buf[:hdr_end], recs, voffs, starts


def aux_items(body):
    """[(tag, type, value bytes)] of a record body."""
    lrn, ncig, lseq = body[8], struct.unpack_from("<H", body, 12)[0], struct.unpack_from("<i", body, 16)[0]
    o = 32 + lrn + 4 * ncig + (lseq + 1) // 2 + lseq
    out = []
    while o < len(body):
        tag, t = body[o:o + 2].decode(), chr(body[o + 2])
        if t in SHORT:
            n = SHORT[t][1]
        elif t == "f":
            n = 4
        elif t == "Z":
            n = body.index(b"\0", o + 3) - (o + 3) + 1
        elif t == "B":
            es = {"c": 1, "C": 1, "s": 2, "S": 2, "i": 4, "I": 4, "f": 4}[chr(body[o + 3])]
            n = 5 + es * struct.unpack_from("<I", body, o + 4)[0]
        else:
            raise ValueError(t)
        out.append((tag, t, body[o + 3:o + 3 + n]))
        o += 3 + n
    return out, 32 + lrn + 4 * ncig + (lseq + 1) // 2 + lseq


def aux_update_int(body, val):
    """htslib bam_aux_update_int(b, "HP", val) restated."""
    if val < -32768 or val > 65535:
        t, sz = ("i" if val < 0 else "I"), 4
    elif val < -128 or val > 255:
        t, sz = ("s" if val < 0 else "S"), 2
    else:
        t, sz = ("c" if val < 0 else "C"), 1
    items, a0 = aux_items(body)
    for k, (tag, ty, v) in enumerate(items):
        if tag != "HP":
            continue
        if ty not in SHORT:
            return body
        old = SHORT[ty][1]
        if old >= sz:
            sz = old
            t = {1: "c", 2: "s", 4: "i"}[old] if val < 0 else {1: "C", 2: "S", 4: "I"}[old]
        items[k] = ("HP", t, struct.pack("<q", val)[:sz])
        break
    else:
        items.append(("HP", t, struct.pack("<q", val)[:sz]))
    return body[:a0] + b"".join(tag.encode() + ty.encode() + v for tag, ty, v in items)


def hp_tag_raw(body):
    """get_hp_from_aln (910-923)."""
    for tag, ty, v in aux_items(body)[0]:
        if tag == "HP":
            if ty not in SHORT:
                return 254
            x = struct.unpack(SHORT[ty][0], v)[0]
            return 254 if x == 0 else x - 1
    return 254


def qname(body):
    return body[32:32 + body[8] - 1].decode()


def _fixture(tmp_path, seed=3):
    rng = random.Random(seed)
    recs = []
    for tid, (lo, hi) in enumerate([(0, 3_000_000), (0, 2_000_000)]):
        for i in range(900):
            pos = rng.randrange(lo, hi)
            lq = rng.randrange(50, 400)
            kind = rng.randrange(9)
            aux = b""
            if kind == 0:
                aux += aux_i("HP", rng.choice([1, 2]))
            elif kind == 1:
                aux += aux_C("HP", rng.choice([1, 2, 3]))
            elif kind == 2:
                aux += aux_Z("HP", "x")
            elif kind == 3:
                aux += struct.pack("<2sch", b"HP", b"s", rng.choice([1, 2, -7]))
            elif kind == 4:
                aux += aux_i("HP", 0)
            elif kind == 5:
                aux += aux_i("HP", 70000)
            aux += aux_f("de", 0.05) + aux_Z("MD", str(lq))
            flag = 4 if rng.random() < 0.02 else 0
            recs.append(Rec(tid, pos, f"q{tid}_{i}", flag=flag, cigar=[(lq << 4) | 0], seq=bytes([0x12] * ((lq + 1) // 2)),
                            l_seq=lq, aux=aux))
    recs.sort(key=lambda r: (r.tid, r.pos))
    big = 70_000                                           # one record larger than a BGZF block
    recs.insert(10, Rec(0, recs[9].pos, "huge", cigar=[(big << 4) | 0], seq=bytes([0x12] * (big // 2)), l_seq=big,
                        aux=aux_i("HP", 1)))
    recs += [Rec(-1, -1, f"u{i}", flag=4, l_seq=10, seq=bytes(5)) for i in range(5)]
    bam = str(tmp_path / "in.bam")
    write_bam(bam, [("c1", 5_000_000), ("c2", 5_000_000)], recs)
    vcf = str(tmp_path / "in.vcf")
    lines = ["##fileformat=VCFv4.2", "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1"]
    for name, gaps in (("c1", [(400_000, 450_000), (1_000_000, 1_020_000), (1_030_000, 1_100_000), (2_000_000, 2_200_000)]),
                       ("c2", [(700_000, 800_000)])):
        tmp = str(tmp_path / f"{name}.vcf")
        write_phased_vcf(tmp, name, gaps)
        lines += [l for l in open(tmp).read().split("\n") if l and not l.startswith("#")]
    open(vcf, "w").write("\n".join(lines) + "\n")
    return recs, bam, vcf


def _restate_methphase(bodies, tids, gaps, blocks, table, raw, tid_names=("c1", "c2")):
    """output_modify_bam (3022-3103) over the input records."""
    out = []
    names = [c["name"] for c in gaps]
    prev_idx, prev_tid, need_flip = 1, 0, 0
    for body, tid in zip(bodies, tids):
        q = qname(body)
        pos = struct.unpack_from("<i", body, 4)[0]
        hp_raw = raw.get(q, 254) if raw is not None else hp_tag_raw(body)
        if tid != prev_tid:
            prev_idx, prev_tid = 1, tid
        c = names.index(tid_names[tid]) if tid >= 0 and tid_names[tid] in names else -1
        updated = False
        if c >= 0:
            g = gaps[c]["gaps"]
            for j in range(prev_idx, len(g)):
                if g[j - 1][1] <= pos <= g[j][0]:
                    if j != prev_idx:
                        updated, prev_idx = True, j
                    break
        if updated:
            fl = blocks[c]["flips"]
            need_flip = fl[prev_idx - 1] if prev_idx - 1 < len(fl) else 0
        if q in table:
            hp = table[q] ^ (1 if need_flip else 0)
        else:
            hp = hp_raw
            if hp in (0, 1) and need_flip:
                hp ^= 1
        out.append(hp)
    return out


@pytest.mark.parametrize("use_raw", [False, True])
def test_write_bam_methphase(tmp_path, use_raw):
    from pomfret_amd import _lib
    from pomfret_amd.bam import RETAG_METHPHASE, BamFile, retag_bam
    from pomfret_amd.pipeline import Tags
    recs, bam, vcf = _fixture(tmp_path)
    g = _lib.Gaps(vcf)
    rng = random.Random(7)
    dec = [rng.choice([-1, 0, 1, 1]) for _ in range(g.n_windows)]
    b = _lib.Blocks(g, dec)
    names = [r.qname for r in recs]
    table = {q: rng.choice([0, 1, 2]) for q in names if rng.random() < 0.3}
    t = Tags()
    t.put_first(list(table), list(table.values()))
    raw, rt = None, None
    if use_raw:
        raw = {q: rng.choice([0, 1, 254]) for q in names if rng.random() < 0.7}
        rt = Tags()
        rt.put_first(list(raw), list(raw.values()))
    out = str(tmp_path / "o.mp.bam")
    n = retag_bam(bam, out, out + ".bai", None, RETAG_METHPHASE, g, b, t, rt)
    assert n == len(recs)
    hi, bodies_in, _, _ = parse_bam(bam)
    ho, bodies_out, voffs, starts = parse_bam(out)
    assert hi == ho and len(bodies_out) == len(bodies_in)
    hp = _restate_methphase(bodies_in, [r.tid for r in recs], g.contigs(), b.contigs(), table, raw)
    for bi, bo, h in zip(bodies_in, bodies_out, hp):
        assert bo == aux_update_int(bi, h + 1)
    # BGZF: the header alone in the first block(s); a record starts a block
    # when it does not fit the current one (bgzf_flush_try)
    blocks = read_bgzf_blocks(out)
    assert len(blocks[0][1]) == len(ho)
    ends = np.cumsum([len(d) for _, d in blocks])
    for v, body in zip(voffs, bodies_out):
        k = int(np.searchsorted(ends, v, side="right"))
        if len(body) + 4 <= 0xff00:
            assert v + 4 + len(body) <= ends[k], "record straddles a block"
    assert blocks[-1][1] == b""
    # the index answers region queries as the overlap rule
    out_recs = [Rec(r.tid, r.pos, r.qname, flag=r.flag, cigar=r.cigar) for r in recs]
    with BamFile(out) as bo_:
        for tid, name in ((0, "c1"), (1, "c2")):
            for s, e in ((100_000, 120_000), (1_500_000, 1_800_000), (0, 10), (2_900_000, 4_000_000)):
                got, qn, _ = bo_.fetch_windows(name, [s], [e], readback=0)
                exp = [out_recs[i].qname for i in expected_fetch(out_recs, tid, s, e, 0)]
                assert qn == exp, (name, s, e)
        assert bo_.index_stats(0)[1] == sum(1 for r in recs if r.tid == 0 and r.flag & 4)


def test_varhaptag_tsv_and_bam(tmp_path):
    from pomfret_amd.bam import RETAG_VARHAPTAG, retag_bam
    from pomfret_amd.pipeline import Tags
    recs, bam, vcf = _fixture(tmp_path, seed=5)
    rng = random.Random(9)
    raw = {r.qname: rng.choice([0, 1, 254]) for r in recs if rng.random() < 0.6}
    rt = Tags()
    rt.put_first(list(raw), list(raw.values()))
    out = str(tmp_path / "v.bam")
    retag_bam(bam, out, out + ".bai", out + ".varhaptag.tsv", RETAG_VARHAPTAG, raw=rt)
    _, bodies_in, _, _ = parse_bam(bam)
    _, bodies_out, _, _ = parse_bam(out)
    lines = open(out + ".varhaptag.tsv").read().split("\n")
    assert lines[0] == "#qname\thaptag_input\thaptag_new" and lines[-1] == ""
    for bi, bo, line in zip(bodies_in, bodies_out, lines[1:-1]):
        h = raw.get(qname(bi), 254)
        assert line == f"{qname(bi)}\t{hp_tag_raw(bi) + 1}\t{h + 1}"
        assert bo == aux_update_int(bi, h + 1)
    # TSV only (varhaptag --write-bam turns the BAM off)
    os.remove(out)
    retag_bam(bam, None, None, out + ".2.tsv", RETAG_VARHAPTAG, raw=rt)
    assert open(out + ".2.tsv").read() == open(out + ".varhaptag.tsv").read() and not os.path.exists(out)


@pytest.mark.parametrize("threads", [2, 3, 8])
def test_write_bam_threads_same_bytes(tmp_path, threads):
    """-T / --bam-threads: the BGZF blocks deflated by a thread pool in batches
    and written in order, the index's virtual offsets taken in block-number
    space and moved to file addresses at the end -- the BAM and the BAI are
    the same bytes as the single-threaded writer's (several batches here), and
    the index answers queries."""
    from pomfret_amd import _lib
    from pomfret_amd.bam import RETAG_METHPHASE, BamFile, retag_bam
    from pomfret_amd.pipeline import Tags
    from tests import _fixtures as fx
    aln, recs, bam, vcf = fx.tagged(tmp_path, n_windows=4)
    g = _lib.Gaps(vcf)
    rng = random.Random(11)
    b = _lib.Blocks(g, [rng.choice([-1, 0, 1]) for _ in range(g.n_windows)])
    table = {r.qname: rng.choice([0, 1]) for r in recs if rng.random() < 0.5}
    t = Tags()
    t.put_first(list(table), list(table.values()))
    outs = []
    for th in (1, threads):
        out = str(tmp_path / f"o{th}.mp.bam")
        n = retag_bam(bam, out, out + ".bai", None, RETAG_METHPHASE, g, b, t, None, threads=th)
        assert n == len(recs)
        outs.append((open(out, "rb").read(), open(out + ".bai", "rb").read()))
    assert len(read_bgzf_blocks(str(tmp_path / "o1.mp.bam"))) > 16 * threads + 2    # more than one batch
    assert outs[0][0] == outs[1][0]
    assert outs[0][1] == outs[1][1]
    with BamFile(str(tmp_path / f"o{threads}.mp.bam")) as bo:
        s, e = int(aln.win_start[1]), int(aln.win_end[1])
        got, qn, _ = bo.fetch_windows("chrS", [s], [e], readback=0)
        assert len(qn) > 0
