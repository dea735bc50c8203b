# Round-5 GPU validation at HEAD (final state: epi2 depth macro, docs test).
set -u -o pipefail
O=gpurun_out/r5ap; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_model_gpu.py -k loss_curve > $O/pytest_curve.log 2>&1 || { tail -30 $O/pytest_curve.log; exit 1; }
tail -2 $O/pytest_curve.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-250
