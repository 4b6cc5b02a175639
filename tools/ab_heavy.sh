# pf_k3_heavy (512 threads, round 6) for the n heaviest problems of the mix
# batch and of its critical window: bash tools/ab_heavy.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
export AB_CACHE=/tmp/ab_aln1024.npz
PF_SYNTH_WORKERS=16 timeout -k 10 300 python3 $R/tools/run_aln_once.py 1024 0 $AB_CACHE 60 > $O/gen.log 2>&1 || exit 13
timeout -k 10 400 python3 -u $R/tools/ab_env.py base: h2:PF_K3_HEAVY=2 h16:PF_K3_HEAVY=16 h64:PF_K3_HEAVY=64 h128:PF_K3_HEAVY=128 h256:PF_K3_HEAVY=256 h512:PF_K3_HEAVY=512 base2: > $O/ab_heavy.txt 2>&1 || exit 14
cat $O/ab_heavy.txt
