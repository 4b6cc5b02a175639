"""Per-loop instruction mix of one kernel in a gfx950 assembly listing
(hipcc --cuda-device-only -S): for every depth-2 loop of the kernel (the
persistent problem loop is depth 1), its instructions with all its child
loops', SALU, LDS, and the SGPR-spill traffic -- v_writelane into, and
v_readlane out of, the VGPRs the compiler spills SGPRs to.

    python tools/isa_loops.py <listing.s> <kernel-name-substring> [top] [depth]

(depth: the loop depth grouped on, 2 by default -- under a persistent loop;
1 for a kernel without one)
"""
import collections
import re
import sys


def kernel_body(lines, name):
    st = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*%s\w*:" % name, l))
    en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    return lines[st:en]


def loop_stats(body, depth=2):
    spillv = {m.group(1) for l in body for m in [re.match(r"\s*v_writelane_b32 (v\d+),", l)] if m}
    top2, stats, hdr = {}, collections.defaultdict(collections.Counter), ("none", 0)
    for i, l in enumerate(body):
        if l.startswith(".LBB") or l.startswith("; %bb"):
            ann, j = [l], i + 1
            while j < len(body) and body[j].strip().startswith(";") and not body[j].startswith("; %bb"):
                ann.append(body[j])
                j += 1
            txt = "\n".join(ann)
            m = re.search(r"in Loop: Header=(BB\d+_\d+) Depth=(\d+)", txt)
            h = re.search(r"Loop Header: Depth=(\d+)", txt)
            if m:
                hdr = (m.group(1), int(m.group(2)))
            elif h:
                lab, d = l.split(":")[0][2:], int(h.group(1))
                hdr = (lab, d)
                if d == depth:
                    top2[lab] = lab
                for p, pd in re.findall(r"Parent Loop (BB\d+_\d+) Depth=(\d+)", txt):
                    if int(pd) == depth:
                        top2[lab] = p
            else:
                hdr = ("none", 0)
            continue
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op, c = s.split()[0], stats[hdr]
        c["instrs"] += 1
        c["salu"] += op.startswith("s_")
        c["lds"] += op.startswith("ds_")
        m = re.match(r"v_readlane_b32 s\w+, (v\d+),", s)
        c["spill_reloads"] += bool(m and m.group(1) in spillv)
        c["spill_stores"] += op == "v_writelane_b32"
    agg = collections.defaultdict(collections.Counter)
    for (h, d), c in stats.items():
        if d >= depth:
            agg[top2.get(h, "?")].update(c)
    return sorted(spillv), agg


if __name__ == "__main__":
    body = kernel_body(open(sys.argv[1]).read().split("\n"), sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    spillv, agg = loop_stats(body, int(sys.argv[4]) if len(sys.argv) > 4 else 2)
    print(f"{sys.argv[2]}: SGPR spill VGPRs {spillv}")
    for h, c in sorted(agg.items(), key=lambda x: -x[1]["instrs"])[:top]:
        print(f"  loop {h:10s} " + " ".join(f"{k} {c[k]}" for k in ("instrs", "salu", "lds", "spill_reloads", "spill_stores")))
