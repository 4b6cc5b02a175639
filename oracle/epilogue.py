"""Output epilogue restated in plain Python -- TEST INFRASTRUCTURE.

Pure-Python loops over small inputs, following the reference line by line
(all line numbers: /root/reference/blockjoin.c):
  lift_decisions                   :2250-2310
  make_decisions_flippings_onraw   :2312-2324
  generate_new_phase_blocks        :2326-2362 (use_raw = 1, as main_blockjoin :4687)
  get_new_phaseblock_ID(1)         :2366-2395
  tmp_check_if_in_dropped_intervals:2397-2409
  get_flip_status                  :2444-2481
  output_tsv / output_gtf          :2696-2756
  alter_vcf_line / output_modify_vcf :2758-2988
Input gaps are the oracle's own window definition (oracle.vcf_gaps, pinned by
the reference's example fixture).  The product is pomfret_amd/csrc/pf_epilogue.c;
only tests/ use this module.

Where the reference reads uninitialised or out-of-range memory this module
takes the same choice as the product (documented there): an unmatched FORMAT
index leaves the line unchanged, an out-of-range flip reads 0, a GT edit past
the end of the rewritten line is skipped.
"""
from __future__ import annotations

import gzip

U32 = 0xFFFFFFFF


def _i32(x):
    x &= U32
    return x - (1 << 32) if x >= 1 << 31 else x


def lift_and_blocks(contig: dict, decisions):
    """One contig: decisions (one per merged gap) -> raw blocks after
    lift_decisions, decisions_onraw, flips_onraw, phase blocks."""
    raw = [list(x) for x in contig["raw"]]
    gaps = contig["gaps"]
    n_raw, n_gap = len(raw), len(gaps)
    # merge_close_intervals: decisions.n = raw count (:2219); ends past the
    # merged count keep their raw values (never overwritten by the merge)
    dec = [int(decisions[i]) if i < n_gap else -1 for i in range(n_raw)]
    ends = [gaps[i][1] if i < n_gap else contig["raw"][i][1] for i in range(n_raw)]
    don = []
    j = 0
    for i in range(n_raw):
        if dec[i] < 0:
            while j < len(raw) and raw[j][1] <= ends[i]:
                don.append(dec[i])
                j += 1
        else:
            if j >= len(raw):
                raise ValueError("lift_decisions: no raw gap left")
            if raw[j][1] < ends[i]:
                j2 = next((k for k in range(j, len(raw)) if raw[k][1] == ends[i]), None)
                if j2 is None:
                    raise ValueError("lift_decisions: assert(found)")
                raw[j][1] = ends[i]
                del raw[j + 1:j2 + 1]
            don.append(dec[i])
            j += 1
    flips, flip = [], 0
    for d in don:
        flip = 0 if d < 0 else flip ^ d
        flips.append(flip)
    blocks = []
    start, end = contig["abs_start"], U32
    for i, d in enumerate(don):
        if d >= 0:
            continue
        end = raw[i][0]
        blocks.append((start, end))
        start = raw[i][1]
    if len(don) > 0 and end != contig["abs_end"]:
        end = contig["abs_start"] if end == U32 else end
        blocks.append((end, contig["abs_end"]))
    return dict(raw=[tuple(x) for x in raw], decisions=don, flips=flips, blocks=blocks)


def phase_blocks(contigs, decisions):
    out, k = [], 0
    for c in contigs:
        n = len(c["gaps"])
        out.append(lift_and_blocks(c, decisions[k:k + n]))
        k += n
    return out


def gtf_text(contigs, blocks) -> str:
    s = []
    for c, b in zip(contigs, blocks):
        for (bs, be) in b["blocks"]:
            bs, be = _i32(bs), _i32(be)
            if bs == 0 or be == 0:
                continue
            s.append(f'{c["name"]}\tPhasing\texon\t{bs}\t{be}\t.\t+\t.\tgene_id "{bs}"; transcript_id "{bs}.1"\n')
    return "".join(s)


def tsv_text(contigs, blocks) -> str:
    return "".join(f'{c["name"]}\t{_i32(bs)}\t{_i32(be)}\n'
                   for c, b in zip(contigs, blocks) for (bs, be) in b["blocks"])


def _sub_idx(s: bytes, idx: int):
    """get_substr_by_idx(s, idx, ':') (:315-337)."""
    start, col = 0, 0
    for i in range(len(s) + 1):
        if i == len(s) or s[i:i + 1] == b":":
            if col == idx:
                return start, i - start
            if i == len(s):
                break
            start, col = i + 1, col + 1
    return None


def _tag_idx(s: bytes, q: bytes):
    """search_substr_idx(s, q, ':', 1, ...) (:283-313)."""
    for col, f in enumerate(s.split(b":")):
        if f == q:
            return col
    return -1


def _atoi(b: bytes) -> int:
    b = b[:20].lstrip(b" \t\n\r\f\v")
    sign, i = 1, 0
    if b[:1] in (b"+", b"-"):
        sign = -1 if b[:1] == b"-" else 1
        i = 1
    v = 0
    while i < len(b) and 48 <= b[i] <= 57:
        v = v * 10 + b[i] - 48
        i += 1
    return _i32(sign * v)


class _VcfState:
    def __init__(self, contigs, blocks, rescue):
        self.contigs, self.blocks, self.rescue = contigs, blocks, rescue
        self.names = [c["name"].encode() for c in contigs]
        self.prev_group_idx = 0
        self.prev_block_idx = 0
        self.last_pos = -1

    def flip_status(self, ci, pos):
        """get_flip_status (:2444-2481)."""
        raw = self.blocks[ci]["raw"]
        flips = self.blocks[ci]["flips"]

        def fl(k):
            return flips[k] if 0 <= k < len(flips) else 0
        j = self.prev_block_idx
        if j >= 0:                 # int j < size_t n: a negative cursor skips the loop
            while j < len(raw):
                start = _i32(raw[j][0])
                if start >= pos:
                    self.prev_block_idx = 0 if j == 0 else j - 1
                    stat = fl(self.prev_block_idx)
                    if (pos & U32) <= raw[0][0]:
                        stat = 0
                    return stat
                j += 1
        self.prev_block_idx = j - 1
        return fl(0 if len(raw) == 0 else len(raw) - 1)

    def alter(self, s: bytes):
        """alter_vcf_line (:2758-2916): (code, new_line)."""
        if s[:1] == b"#":
            if s[1:2] == b"#":
                return 0, None
            if s.count(b"\t") + 1 != 10:
                raise ValueError("vcf header column count")
            return 0, None
        col, start, pos, i_ps, i_gt, ci = 0, 0, 0, -1, -1, None
        for i in range(len(s)):
            if s[i:i + 1] != b"\t":
                continue
            if col == 0:
                name = s[start:i]
                ci = self.names.index(name) if name in self.names else None
                pos, i_ps, i_gt = 0, -1, -1
                if ci is None:
                    break
            elif col == 1:
                pos = _atoi(s[start:i])
                if pos < self.last_pos:
                    self.prev_group_idx = 0
                    self.prev_block_idx = 0
                self.last_pos = pos
            elif col == 8:
                fmt = s[start:i] if i > start else s[start:]
                i_ps = _tag_idx(fmt, b"PS")
                i_gt = _tag_idx(fmt, b"GT")
            col += 1
            start = i + 1
        if pos == 0 or i_ps < 0:
            return 0, None
        smp = s[start:]
        ps = _sub_idx(smp, i_ps)
        gt = _sub_idx(smp, i_gt) if i_gt >= 0 else None
        if ps is None or gt is None:
            return 0, None
        ps_s, ps_l = ps
        gt_s, gt_l = gt
        if ps_l == 1 and smp[ps_s:ps_s + 1] == b".":
            return 0, None
        GT = smp[gt_s:gt_s + min(gt_l, 9)] + b"\0\0\0"
        if GT[1:2] != b"|" or GT[0:1] not in (b"0", b"1") or GT[2:3] not in (b"0", b"1"):
            return 0, None
        group = -1
        for k, (bs, be) in enumerate(self.blocks[ci]["blocks"]):
            if bs == U32 or be == 0 or be == U32:
                continue
            if bs <= (pos & U32) < be:
                self.prev_group_idx = k
                group = _i32(bs)
                break
        dropped = any(ds <= (pos & U32) <= de for (ds, de) in self.contigs[ci]["dropped"])
        need_flip = self.flip_status(ci, pos)
        middle = False
        if group >= 0 and dropped and self.rescue is not None:
            h = self.rescue[ci].get((pos - 1) & U32, -1)
            middle = h in (0, 1)
        off = start + ps_s
        if group < 0 or dropped:
            if not middle:
                return 0, None
            nl = bytearray(s[:off] + b"." + s[off + ps_l:])
            if start + gt_s + 1 < len(nl):
                nl[start + gt_s + 1] = ord("/")
            return 2, bytes(nl)
        nl = bytearray(s[:off] + str(group).encode() + s[off + ps_l:])
        if need_flip:
            a = start + gt_s
            if a < len(nl):
                nl[a] = ord("1") if nl[a] == ord("0") else ord("0")
            if a + 2 < len(nl):
                nl[a + 2] = ord("1") if nl[a] == ord("0") else ord("0")
        return 1, bytes(nl)


def vcf_bytes(vcf_in: str, contigs, blocks, rescue=None):
    """output_modify_vcf: (rewritten VCF bytes, (modified, unphased, lines))."""
    with open(vcf_in, "rb") as f:
        raw = f.read()
    if raw[:2] == b"\x1f\x8b":
        raw = gzip.decompress(raw)
    st = _VcfState(contigs, blocks, rescue)
    out, n_mod, n_drop, n_tot = [], 0, 0, 0
    lines = raw.split(b"\n")[:-1]          # a final line without '\n' is never processed
    for line in lines:
        code, nl = st.alter(line)
        n_tot += 1
        if code == 0:
            out.append(line + b"\n")
        else:
            n_drop += code == 2
            n_mod += code == 1
            out.append(nl + b"\n")
    return b"".join(out), (n_mod, n_drop, n_tot)
