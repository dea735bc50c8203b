# Round-5 GPU checks, part s: refresh the README's secondary bench rows at HEAD.
set -u -o pipefail
O=gpurun_out/r5s; mkdir -p $O
b() { local n=$1; shift; timeout -k 10 600 python bench.py "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }; echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("peak_mem_gib"))')"; }
b gpt2m_b16 --model gpt2-medium --batch-per-gpu 16 --steps 20 --warmup 5
b llama3_8b_s2048_b16 --model llama3-8b --batch-per-gpu 16 --steps 10 --warmup 3
b llama3_8b_s2048_b1 --model llama3-8b --batch-per-gpu 1 --steps 30 --warmup 5
b llama2_7b_b1 --model llama2-7b --batch-per-gpu 1 --steps 30 --warmup 5
