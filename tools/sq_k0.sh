# SQ counter passes over the record-level batch (K0 diagnosis), run on the GPU box:
#   bash tools/sq_k0.sh <outdir>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-sqk0}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/run_aln_once.py 256 0 /tmp/aln256.npz || exit 20
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $O/p1 -o p1 --output-format csv -- python3 $R/tools/run_aln_once.py 256 2 /tmp/aln256.npz > $O/p1.log 2>&1 || exit 21
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD -d $O/p2 -o p2 --output-format csv -- python3 $R/tools/run_aln_once.py 256 2 /tmp/aln256.npz > $O/p2.log 2>&1 || exit 22
echo done
