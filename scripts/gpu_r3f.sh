# round 3: full GPU suite on the current tree (+ f3 worst case timing)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-r3f}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?
cp gpurun_out/f3_worst_case.json gpurun_out/$T/ 2>/dev/null
exit $rc
