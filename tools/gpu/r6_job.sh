#!/bin/bash
# Round 6 file-job check: ingest GPU tests, then the y4m job with SDMA ingest and with HIP
# copies (alternating), then the synthetic job.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r6job}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ingest.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
one() { n=$1; shift; timeout -k 10 600 env "$@" python -u bench.py --job --source y4m > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 30 $O/$n.log; exit 1; }
  python3 -c "import json; r=json.loads([l for l in open('$O/$n.log') if l.startswith('{')][-1]); c=r['config']; s=c['rank0_spans_ms']; print('$n', r['value'], 'encode ms/claim', s['node_job.encode']['avg_ms'], 'load max', s['node_job.load']['max_ms'], c['per_rank_ingest'][0]['ingest_gb_per_s'])"; }
one sdma1 TV_NOP=1 && one hip1 TV_INGEST_DMA=hip && one sdma2 TV_NOP=1 && one hip2 TV_INGEST_DMA=hip
timeout -k 10 600 python -u bench.py --job > $O/job_synth.log 2>&1 || { echo "synth job failed"; tail -n 30 $O/job_synth.log; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('$O/job_synth.log') if l.startswith('{')][-1]); print('synth', r['value'])"
