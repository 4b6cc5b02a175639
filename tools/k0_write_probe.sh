# K0 write traffic by phase: WRITE_SIZE passes with PF_K0_DIAG = 2 / 3 / 0
# (stop after MM / after the SEQ pass / whole kernel) on 256 windows (50 kb)
#   bash tools/k0_write_probe.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-k0w}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PF_SYNTH_WORKERS=16 timeout -k 10 200 python3 $R/tools/run_aln_once.py 256 0 /tmp/a256.npz 60 fixed50 > $O/gen.log 2>&1 || exit 10
for M in 2 3 0; do
  PF_K0_DIAG=$M timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w$M -o w$M --output-format csv -- python3 $R/tools/run_aln_once.py 256 2 /tmp/a256.npz 60 fixed50 > $O/w$M.log 2>&1 || exit 11
  PF_K0_DIAG=$M timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f$M -o f$M --output-format csv -- python3 $R/tools/run_aln_once.py 256 2 /tmp/a256.npz 60 fixed50 > $O/f$M.log 2>&1 || exit 12
done
rm -f /tmp/a256.npz
for M in 2 3 0; do
  python3 - $O/w$M/w${M}_counter_collection.csv $O/f$M/f${M}_counter_collection.csv $M <<'PY'
import csv, sys, collections
def agg(p, c):
    v = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        if r["Counter_Name"] == c and r["Kernel_Name"].startswith("pf_k0_load"):
            v[r["Dispatch_Id"]].append(float(r["Counter_Value"]))
    s = [sum(x) for x in v.values()]
    return sum(s) / len(s) / 1e6 if s else 0
print(f"PF_K0_DIAG={sys.argv[3]}: K0 WRITE {agg(sys.argv[1], 'WRITE_SIZE'):.3f} GB  FETCH(x2) {2 * agg(sys.argv[2], 'FETCH_SIZE'):.3f} GB (KiB/1e6)")
PY
done
