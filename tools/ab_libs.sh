# A/B of library builds on the bench's mix batch (tools/ab_env.py via
# tools/ab_lib.py), the batch generated once before any GPU work:
#   bash tools/ab_libs.sh <tag> libpomfret_amd.so libpomfret_amd_v1.so ...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
shift
mkdir -p $O
export AB_CACHE=/tmp/ab_aln1024.npz
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 $R/tools/run_aln_once.py 1024 0 $AB_CACHE 60 > $O/gen.log 2>&1 || exit 13
for lib in "$@"; do
  echo "== $lib" | tee -a $O/ab.txt
  timeout -k 10 400 python3 -u $R/tools/ab_lib.py $lib ${AB_CONFIGS:-base:} >> $O/ab.txt 2>&1 || exit 14
done
cat $O/ab.txt
