#!/bin/bash
# DVD job (MPEG-2 480i MKV -> bwdif -> HEVC): plain run, then a kernel summary of it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-dvdprof}; mkdir -p $O
timeout -k 10 300 python -u bench.py --job --source mpeg2 > $O/dvd.log 2>&1
rc=$?; echo "dvd rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/dvd.log; exit $rc; }
grep '^{' $O/dvd.log | tail -1 | python3 -c "import json,sys; r=json.load(sys.stdin); c=r['config']; print(r['value'], c['rank0_spans_ms'])"
[ -n "$NOPROF" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --job --source mpeg2 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof.log; exit $rc; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 16 | tee $O/kernel_summary.txt
