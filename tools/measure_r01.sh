set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${MEAS_TAG:-m3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 $R/bench.py --no-cpu --steps 20 > $O/bench_prof.json 2> $O/bench_prof.err || exit 12
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 $R/tools/run_once.py 30 3 > $O/fetch.log 2>&1 || exit 13
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 $R/tools/run_once.py 30 3 > $O/write.log 2>&1 || exit 14
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/calf -o calf --output-format csv -- $R/tools/ubench/hbm_cal > $O/calf.log 2>&1 || exit 15
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/calw -o calw --output-format csv -- $R/tools/ubench/hbm_cal > $O/calw.log 2>&1 || exit 16
echo done
