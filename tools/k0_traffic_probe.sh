# K0 HBM traffic by phase on the bench's mix batch (1024 windows, 60x): FETCH_SIZE
# and WRITE_SIZE passes with PF_K0_DIAG = 4 / 2 / 5 / 3 / 0 (stop after the
# filters / the MM phase / the SEQ count / the SEQ pass / the whole kernel),
# the batch generated before any profiler starts.
#   bash tools/k0_traffic_probe.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-k0t}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 $R/tools/run_aln_once.py 1024 0 /tmp/a1024.npz 60 > $O/gen.log 2>&1 || exit 10
for M in 4 2 5 3 0; do
  PF_K0_DIAG=$M timeout -k 10 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w$M -o w$M --output-format csv -- python3 $R/tools/run_aln_once.py 1024 2 /tmp/a1024.npz 60 > $O/w$M.log 2>&1 || exit 11
  PF_K0_DIAG=$M timeout -k 10 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f$M -o f$M --output-format csv -- python3 $R/tools/run_aln_once.py 1024 2 /tmp/a1024.npz 60 > $O/f$M.log 2>&1 || exit 12
  echo "diag $M done"
done
rm -f /tmp/a1024.npz
for M in 4 2 5 3 0; do
  python3 - $O/w$M/w${M}_counter_collection.csv $O/f$M/f${M}_counter_collection.csv $M <<'PY' | tee -a $O/summary.txt
import csv, sys, collections
def agg(p, c):
    v = collections.defaultdict(float)
    for r in csv.DictReader(open(p)):
        if r["Counter_Name"] == c and r["Kernel_Name"].startswith("pf_k0_load"):
            v[r["Dispatch_Id"]] += float(r["Counter_Value"])
    s = list(v.values())
    return sum(s) / len(s) * 1024 / 1e9 if s else 0
w, f = agg(sys.argv[1], "WRITE_SIZE"), 2 * agg(sys.argv[2], "FETCH_SIZE")
print(f"PF_K0_DIAG={sys.argv[3]}: K0 read {f:.3f} GB  written {w:.3f} GB  total {f + w:.3f} GB per launch")
PY
done
