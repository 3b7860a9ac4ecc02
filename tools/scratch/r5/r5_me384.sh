set -o pipefail
export TV_HIPFLAGS_EXTRA="-DTV_ME_THREADS=384" PYTHONPATH=$PWD TMPDIR=/tmp TV_NO_AUTOBUILD=1
O=gpurun_out/me384; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_scenecut.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
TV_ENGINE_GROUPS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g1 -o run -- python3 bench.py --no-4k --steps 2 --warmup 1 > $O/g1.log 2>&1 || exit 1
python3 tools/kstats.py $(find $O/g1 -name "*kernel_stats.csv" | head -1) 40 | grep -E "k_inter_me|k_inter_recon"
for k in 1 2; do timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-4k > $O/bench$k.log 2>&1 || exit 1; grep "^{" $O/bench$k.log | cut -c1-120; done
