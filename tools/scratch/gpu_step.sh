set -o pipefail
TAG=${1:-step}; shift
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_scenecut.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/$TAG/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 "$@" > gpurun_out/$TAG/bench.log 2>&1; rc=$?; tail -1 gpurun_out/$TAG/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- python3 bench.py --steps 2 --warmup 1 "$@" > gpurun_out/$TAG/prof.log 2>&1 || exit 1
python3 tools/profsum.py $(find gpurun_out/$TAG/prof -name "*kernel_trace.csv" | head -1) --skip 0.5 | head -16
