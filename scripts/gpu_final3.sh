# final tree: smoke, GPU tests, bench (N=1), two-rank rehearsal on one GPU, rocprof trace of the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r2_final3}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err && \
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/$T/bench_n2.json 2> gpurun_out/$T/bench_n2.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/trace -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/$T/trace_bench.json 2> gpurun_out/$T/trace_bench.err && \
python3 scripts/trace_summary.py gpurun_out/$T/trace/run_kernel_trace.csv 20 > gpurun_out/$T/trace_summary.json
