# Round-6 probe on the GPU box: new tests, the K0 A/B (waves per SIMD), and
# K0's instruction-cache counters.
#   bash tools/r06_probe.sh <tag> [pytest selection]
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r06p}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $2 > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 11; }
  tail -3 $O/pytest.log
fi
bash tools/ab_libs.sh $T/ab ${AB_LIBS:-libpomfret_amd.so} || exit 12
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*" $O/avail.txt | sort -u > $O/icache_counters.txt
echo "icache counters: $(cat $O/icache_counters.txt | tr '\n' ' ')"
C=$(grep -x "SQC_ICACHE_MISSES\|SQC_ICACHE_HITS\|SQ_IFETCH" $O/icache_counters.txt | tr '\n' ' ')
if [ -n "$C" ]; then
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C SQ_WAVES -d $O/ic -o ic --output-format csv -- python3 $R/tools/run_aln_once.py 1024 2 /tmp/ab_aln1024.npz 60 > $O/ic.log 2>&1 || exit 13
  echo "icache pass done"
fi
