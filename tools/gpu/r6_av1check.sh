#!/bin/bash
# Round 6: AV1 engine check -- AV1 GPU tests (golden / dav1d), two AV1 4K benches and a
# kernel trace of the AV1 4K pass.  Usage: r6_av1check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-r6av1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -k "av1" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 600 python -u bench.py --codec av1 --res 4k --steps 4 --warmup 2 > $O/b$r.log 2>&1 || { echo "bench failed"; tail -n 5 $O/b$r.log; exit 1; }
  python3 -c "import json; L=[l for l in open('$O/b$r.log') if l.startswith('{')]; r=json.loads(L[-1]); print('av1_4k', r['value'], r['config'].get('psnr_y_db'), r['config'].get('kbps_per_30fps_stream'))"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g1 -o run -- python3 bench.py --codec av1 --res 4k --steps 2 --warmup 1 > $O/g1.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/profsum.py $(find $O/g1 -name "*kernel_trace.csv" | head -1) --skip 0.4 > $O/g1_summary.txt 2>&1; head -n 10 $O/g1_summary.txt
