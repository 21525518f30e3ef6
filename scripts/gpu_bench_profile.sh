set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --maxit 50 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --maxit 50 --no-cpu > gpurun_out/prof1.log 2>&1
echo EXIT $?
cat gpurun_out/bench_small.json; tail -5 gpurun_out/bench_small.err
find gpurun_out/prof1 -name "*stats*" | head; 
