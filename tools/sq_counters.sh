# SQ counter passes over the bench workload (K3 diagnosis), run on the GPU box:
#   bash tools/sq_counters.sh <outdir>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-sq}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $O/p1 -o p1 --output-format csv -- python3 $R/tools/run_once.py 30 3 > $O/p1.log 2>&1 || exit 21
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d $O/p2 -o p2 --output-format csv -- python3 $R/tools/run_once.py 30 3 > $O/p2.log 2>&1 || exit 22
echo done
