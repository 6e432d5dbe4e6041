# A/B call: smoke + GPU tests (optional) + read probes + kernel variants, each under its own limit
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-ab}
mkdir -p gpurun_out/$T
if [ -n "$WITH_TESTS" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 && \
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || exit $?
fi
timeout -k 10 ${AB_TIMEOUT:-300} python -u scripts/ab.py ${AB_WORK:-zipf} ${AB_VARIANTS:-0} > gpurun_out/$T/ab.jsonl 2> gpurun_out/$T/ab.err
