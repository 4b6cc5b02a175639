"""Device BGZF inflate (pf_inflate.hip) against zlib on BGZF blocks of every
DEFLATE form: stored, fixed and dynamic Huffman blocks, every zlib strategy,
several deflate blocks per BGZF block, long matches, empty blocks, the
BAM files the test writer makes, and corrupted blocks (CRC, truncation)."""
import os
import struct
import zlib

import numpy as np
import pytest

from tests import _bamio

pytestmark = pytest.mark.gpu


def bgzf_block(data: bytes, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, mem=8) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, -15, mem, strategy)
    z = c.compress(data) + c.flush()
    bsize = 18 + len(z) + 8
    if bsize > 65536:                    # htslib shrinks such an input; not a valid block
        return None
    hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize - 1)
    return hdr + z + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


def payloads(rng):
    out = [b"", b"a", bytes(65536), bytes(range(256)) * 256]
    out.append(rng.integers(0, 256, 65536, dtype=np.uint8).tobytes())           # incompressible
    out.append(rng.integers(0, 4, 65536, dtype=np.uint8).tobytes())             # 2-bit alphabet
    q = rng.normal(20, 6, 60000).clip(2, 50).astype(np.uint8).tobytes()        # quality-like
    out.append(q)
    txt = b"".join(b"C+m?,%d,%d;" % (rng.integers(0, 30), rng.integers(0, 300)) for _ in range(5000))[:65536]
    out.append(txt)
    base = rng.integers(0, 256, 3000, dtype=np.uint8).tobytes()
    out.append((base * 30)[:65536])                                           # distances ~3000
    out.append(b"ab" * 30000 + b"xyz" * 1000)                                  # overlapping short matches
    for n in (1, 2, 3, 7, 255, 256, 257, 4095, 65280):
        out.append(rng.integers(0, 3, n, dtype=np.uint8).tobytes())
    return [p[:65280] for p in out]          # BGZF_BLOCK_SIZE: a block's input never exceeds 0xff00


def test_inflate_forms(gpu_ctx):
    rng = np.random.default_rng(7)
    pl = payloads(rng)
    modes = [(0, zlib.Z_DEFAULT_STRATEGY, 8), (1, zlib.Z_DEFAULT_STRATEGY, 8), (6, zlib.Z_DEFAULT_STRATEGY, 8),
             (9, zlib.Z_DEFAULT_STRATEGY, 9), (6, zlib.Z_FIXED, 8), (6, zlib.Z_HUFFMAN_ONLY, 8),
             (6, zlib.Z_RLE, 8), (6, zlib.Z_FILTERED, 8), (5, zlib.Z_DEFAULT_STRATEGY, 1)]   # mem 1: many deflate blocks
    comp = bytearray()
    want = bytearray()
    for i, p in enumerate(pl):
        for lv, stg, mem in modes:
            blk = bgzf_block(p, lv, stg, mem)
            if blk is None:
                continue
            comp += blk
            want += p
    got, st, ms = gpu_ctx.bgzf_inflate(bytes(comp))
    assert not st.any()
    assert got == bytes(want)


def test_inflate_bam_file(gpu_ctx, tmp_path):
    from pomfret_amd.synth_aln import AlnSpec, make_aln_batch
    aln = make_aln_batch(AlnSpec(n_windows=2, coverage=30, seed=3, len_scale=0.5), workers=1)
    recs = _bamio.records_from_aln(aln)
    path = str(tmp_path / "x.bam")
    _bamio.write_bam(path, [("chrS", 2_000_000_000)], recs)
    data = open(path, "rb").read()
    got, st, ms = gpu_ctx.bgzf_inflate(data)
    want = bytearray()
    o = 0
    while o < len(data):
        bsize = struct.unpack_from("<H", data, o + 16)[0] + 1
        want += zlib.decompress(data[o + 18:o + bsize - 8], -15)
        o += bsize
    assert got == bytes(want)


def test_inflate_errors(gpu_ctx):
    from pomfret_amd._lib import PomfretError
    rng = np.random.default_rng(1)
    good = bgzf_block(rng.integers(0, 4, 50000, dtype=np.uint8).tobytes())
    bad_crc = bytearray(good)
    bad_crc[-8] ^= 1
    with pytest.raises(PomfretError):
        gpu_ctx.bgzf_inflate(good + bytes(bad_crc) + good)
    assert list(gpu_ctx.last_inflate_status[:3]) == [0, 7, 0]
    bad_size = bytearray(good)
    struct.pack_into("<I", bad_size, len(bad_size) - 4, 49999)
    with pytest.raises(PomfretError):
        gpu_ctx.bgzf_inflate(bytes(bad_size))
    assert gpu_ctx.last_inflate_status[0] == 5
    # garbage payload: must fail (any code), never hang or write out of bounds
    junk = bytearray(good)
    junk[18:18 + 200] = rng.integers(0, 256, 200, dtype=np.uint8).tobytes()
    with pytest.raises(PomfretError):
        gpu_ctx.bgzf_inflate(bytes(junk) + good)
    assert gpu_ctx.last_inflate_status[0] != 0 and gpu_ctx.last_inflate_status[1] == 0


def test_inflate_throughput(gpu_ctx):
    """Many blocks at once (bench-like): BAM-like content (4-bit SEQ + a
    quality string), timed; the blocks reuse a few payloads so the test stays
    quick to build."""
    rng = np.random.default_rng(3)
    kinds = []
    for i in range(16):
        seq = rng.integers(0, 16, 20000, dtype=np.uint8)
        seqb = (seq[0::2] << 4 | seq[1::2]).astype(np.uint8).tobytes()
        q = rng.normal(20, 6, 45536).clip(2, 50).astype(np.uint8).tobytes()
        d = (seqb + q)[:65280]
        kinds.append((d, bgzf_block(d, 6)))
    n = 8192
    comp = b"".join(kinds[i % 16][1] for i in range(n))
    raw = sum(len(kinds[i % 16][0]) for i in range(n))
    got, st, ms = gpu_ctx.bgzf_inflate(comp)
    assert not st.any() and len(got) == raw
    assert got[:len(kinds[0][0]) + len(kinds[1][0])] == kinds[0][0] + kinds[1][0]
    print(f"\n[inflate] {n} blocks, {raw / 1e6:.0f} MB out, {len(comp) / 1e6:.0f} MB in: "
          f"{ms:.3f} ms = {raw / ms / 1e6:.1f} GB/s")
