set -o pipefail
O=gpurun_out/s1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
bash tools/bench_final.sh s1
