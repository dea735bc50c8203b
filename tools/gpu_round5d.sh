# Round-5 GPU checks, part d: hardware queues per process (GPU_MAX_HW_QUEUES) vs stream sharing.
set -u
O=gpurun_out/r5d; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for q in 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 rocprofv3 --kernel-trace -d $O/qprobe$q -o q -- python3 tools/queue_probe.py > $O/qprobe$q.log 2>&1 || { tail -20 $O/qprobe$q.log; exit 1; }
  python tools/queue_probe.py --summary $(find $O/qprobe$q -name 'q_results.db' | head -1) > $O/queue_map$q.md 2>&1; cat $O/queue_map$q.md
done
for r in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_q${q}_r$r.log 2>&1 || exit 1
    echo "queues=$q round=$r $(tail -1 $O/bench_q${q}_r$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
