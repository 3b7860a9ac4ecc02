#!/bin/bash
# AV1 worker-path tests + AV1 end-to-end job bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-av1_job}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_av1_codec.py tests/test_av1_conformance.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --job --codec av1 > $O/job_av1.log 2>&1 || { echo "job failed"; tail -n 8 $O/job_av1.log; exit 1; }
python -c "import json; r=json.loads([l for l in open('$O/job_av1.log') if l.startswith('{')][-1]); c=r['config']; print('job_av1', r['value'], c.get('psnr_y_db'), c['rank0_spans_ms']['node_job.encode'])"
