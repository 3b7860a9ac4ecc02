#!/bin/bash
# AV1 iteration: AV1 GPU tests (GPU == golden, dav1d conformance), then the 1080p / 4K benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-av1_iter}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_av1_codec.py tests/test_av1_conformance.py tests/test_av1_tools.py tests/test_av1_deblock.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1080p 4k; do
  timeout -k 10 400 python -u bench.py --codec av1 --res $r --steps 4 --warmup 2 > $O/bench_$r.log 2>&1 || { echo "bench $r failed"; tail -n 5 $O/bench_$r.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('$O/bench_$r.log') if l.startswith('{')][-1]); print('$r', r['value'], r['config']['psnr_y_db'], r['config']['kbps_per_30fps_stream'])"
done
