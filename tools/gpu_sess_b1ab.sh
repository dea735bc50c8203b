export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 240 env "$@" python -u bench.py --batch-per-gpu 1 --steps 30 --warmup 5 $EXTRA > gpurun_out/b1_$name.log 2>&1 || { tail -20 gpurun_out/b1_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/b1_$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
EXTRA="" run default A=1
EXTRA="--no-overlap-optimizer" run no_overlap A=1
EXTRA="" run no_shadows PRA_WEIGHT_SHADOWS=0
EXTRA="" run wgrad_hip PYRECOVER_WGRAD=hip
EXTRA="" run default2 A=1
