# Round-5 GPU checks, part c: communication prediction, hardware-queue map, other configs.
set -u
O=gpurun_out/r5c; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/comm_predict.py --model llama2-7b --batch-per-gpu 16 --json $O/comm_predict_7b_b16.json > $O/comm_predict_7b_b16.log 2>&1 || { tail -20 $O/comm_predict_7b_b16.log; exit 1; }
timeout -k 10 300 python tools/comm_predict.py --model llama3-8b --batch-per-gpu 1 --steps 6 --json $O/comm_predict_8b_b1.json > $O/comm_predict_8b_b1.log 2>&1 || { tail -20 $O/comm_predict_8b_b1.log; exit 1; }
grep -v '^{' $O/comm_predict_*.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/qprobe -o q -- python3 tools/queue_probe.py > $O/qprobe.log 2>&1 || { tail -20 $O/qprobe.log; exit 1; }
python tools/queue_probe.py --summary $(find $O/qprobe -name 'q_results.db' | head -1) > $O/queue_map.md 2>&1; cat $O/queue_map.md
timeout -k 10 300 python bench.py --model llama3-8b --batch-per-gpu 1 --steps 20 --warmup 5 > $O/bench_8b_b1.log 2>&1 || exit 1
tail -1 $O/bench_8b_b1.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "streamk or dkdv" > $O/pytest_streamk.log 2>&1 || { tail -20 $O/pytest_streamk.log; exit 1; }
tail -1 $O/pytest_streamk.log
timeout -k 10 300 python tools/wgrad_bench.py --rounds 3 > $O/wgrad_bench_7b_hybrid.log 2>&1 || exit 1
grep shape $O/wgrad_bench_7b_hybrid.log
