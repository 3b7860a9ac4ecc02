#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
bash tools/gpu/ab_env.sh r6_multi/grp4k TV_NOP=1 TV_ENGINE_GROUPS=3 --res 4k || exit 1
bash tools/gpu/ab_env.sh r6_multi/grpent TV_NOP=1 TV_ENGINE_GROUPS=3 --no-4k --entropy gpu || exit 1
bash tools/gpu/r6_av1.sh r6_multi/av1
