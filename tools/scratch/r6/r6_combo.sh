#!/bin/bash
# Round 6 combined session: engine + entropy golden tests, SDMA-vs-HIP D2H A/B, packed-SAO
# A/B, stream-group A/B, then the GPU-CABAC bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
T=${1:-r6combo}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_entropy.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab_env.sh $T/d2h TV_NOP=1 TV_D2H=hip --no-4k || exit 1
bash tools/gpu/ab_env.sh $T/sao TV_NOP=1 TV_SAO_PACKED=0 --no-4k || exit 1
bash tools/gpu/ab_env.sh $T/grp TV_NOP=1 TV_ENGINE_GROUPS=3 --no-4k || exit 1
timeout -k 10 300 python -u bench.py --no-4k --steps 6 --warmup 2 --entropy gpu > $O/gpuent.log 2>&1 || { echo "gpuent failed"; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('$O/gpuent.log') if l.startswith('{')][-1]); print('gpu entropy', r['value'], r['config']['per_rank_cpu'][0]['busy_cores'])"
