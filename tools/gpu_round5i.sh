# Round-5 GPU checks, part i: fused attention backward in pytest and in the 7B B16 step.
set -u -o pipefail
O=gpurun_out/r5i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -2 $O/pytest_attn.log
timeout -k 10 600 python tools/step_ab.py --rounds 3 --steps 4 --arm "split:attn.bwd_fused=0" --arm "fused:attn.bwd_fused=1" > $O/step_ab_fused_bwd.log 2>&1 || { tail -30 $O/step_ab_fused_bwd.log; exit 1; }
grep median $O/step_ab_fused_bwd.log
