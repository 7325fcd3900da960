#!/bin/bash
# One gpurun call: GPU tests, smoke, 1-GPU bench, 2-rank plumbing bench (both ranks on cuda:0,
# gloo). Stops at the first step that faults / aborts / times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/summary.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/summary.log
  tail -4 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
: > gpurun_out/summary.log
for step in ${STEPS_TO_RUN:-pytest smoke bench share2}; do
  case $step in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 8 ;;
    share2) run share2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
              --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 2 \
              --batch 64 --share-gpu --backend gloo ;;
    savedb) tar -C . -czf gpurun_out/miopen_cache.tgz .miopen && ls -la gpurun_out/miopen_cache.tgz ;;
    prof) run prof 900 bash scripts/prof_step.sh ${PROF_TAG:-step} ;;
  esac
done
echo done
