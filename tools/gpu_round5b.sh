set -u
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_attention_shapes_gpu.py tests/test_xgmi_gpu.py -k "attention or attn or wgrad or xgmi or rccl" > $O/pytest_attn_wgrad.log 2>&1 || { tail -30 $O/pytest_attn_wgrad.log; exit 1; }
tail -2 $O/pytest_attn_wgrad.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_7b_b16.log 2>&1 || exit 1
tail -1 $O/bench_7b_b16.log
timeout -k 10 300 python tools/wgrad_bench.py --rounds 3 > $O/wgrad_bench_7b.log 2>&1 || exit 1
timeout -k 10 300 python tools/wgrad_bench.py --rounds 3 --tokens 2048 --dims qkv:6144:4096,o:4096:4096,w13:28672:4096,w2:4096:14336,head:128256:4096 > $O/wgrad_bench_8b_b1.log 2>&1 || exit 1
grep shape $O/wgrad_bench_*.log
timeout -k 10 400 python tools/step_ab.py --arm "ring:attn.dkdv_kreg=2" --arm "lds:attn.dkdv_kreg=0" --rounds 3 --steps 5 > $O/step_ab_ring.log 2>&1 || exit 1
grep median $O/step_ab_ring.log
timeout -k 10 400 python tools/step_ab.py --model llama3-8b --batch-per-gpu 1 --arm "base:" --arm "hipwg:ops.fused.WGRAD_AUTO_MIN_TOKENS=2048" --arm "hipwgsk:ops.fused.WGRAD_AUTO_MIN_TOKENS=2048;wgrad.streamk=1" --rounds 3 --steps 10 > $O/step_ab_8b_b1_wgrad.log 2>&1 || exit 1
grep median $O/step_ab_8b_b1_wgrad.log
