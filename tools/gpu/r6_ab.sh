#!/bin/bash
# Round 6: generic same-box A/B -- engine golden tests, then bench pairs A (default) / B (the
# given env assignment) x 2, then a single-group kernel trace of A.  Usage: r6_ab.sh <tag> VAR=value
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-r6ab}; BENV=${2:-TV_NOP=1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_bframes.py tests/test_gpu_entropy.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
val() { python3 -c "import json; L=[l for l in open('$1') if l.startswith('{')]; r=json.loads(L[-1]); print(r['value'], r['config'].get('fps_4k'), r['config'].get('psnr_y_db'), r['config'].get('kbps_per_30fps_stream'))"; }
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/b_A$r.log 2>&1 || { echo "bench A failed"; tail -n 5 $O/b_A$r.log; exit 1; }
  echo "A$r $(val $O/b_A$r.log)"
  env $BENV timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/b_B$r.log 2>&1 || { echo "bench B failed"; tail -n 5 $O/b_B$r.log; exit 1; }
  echo "B$r $(val $O/b_B$r.log)"
done
TV_ENGINE_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g1 -o run -- python3 bench.py --no-4k --steps 3 --warmup 1 > $O/g1.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/profsum.py $(find $O/g1 -name "*kernel_trace.csv" | head -1) --skip 0.4 > $O/g1_summary.txt 2>&1; head -n 10 $O/g1_summary.txt
