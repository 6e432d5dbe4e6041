set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/${TAG:-r1}_smi.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-r1}_smoke.log 2>&1 && \
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG:-r1}_pytest_gpu.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG:-r1}_bench.json 2> gpurun_out/${TAG:-r1}_bench.err
