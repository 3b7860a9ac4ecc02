#!/bin/bash
# Round 6 file-job check: the y4m job (direct) and the synthetic job, default settings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r6job}; mkdir -p $O
timeout -k 10 600 python -u bench.py --job --source y4m > $O/job_y4m.log 2>&1 || { echo "y4m failed"; tail -n 30 $O/job_y4m.log; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('$O/job_y4m.log') if l.startswith('{')][-1]); c=r['config']; print('y4m', r['value'], {k: c.get(k) for k in ('claims','per_rank_ingest','engine_fps','encode_ms_per_claim','stage_s') if k in c})"
timeout -k 10 600 python -u bench.py --job > $O/job_synth.log 2>&1 || { echo "synth job failed"; tail -n 30 $O/job_synth.log; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('$O/job_synth.log') if l.startswith('{')][-1]); print('synth', r['value'])"
