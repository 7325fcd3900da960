# Same process configuration twice (tuners off: fixed kernels): the 300-step accuracy runs must
# agree bit for bit (every loss / top-1 value).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  LWAAAI_GEMM_TUNE=0 LWAAAI_CONV_TUNE=0 timeout -k 10 300 python scripts/accuracy_r50.py > gpurun_out/det_$i.jsonl 2>&1 || { tail gpurun_out/det_$i.jsonl; exit 1; }
done
grep -h '^{' gpurun_out/det_1.jsonl | python -c "import sys,json; [print(json.loads(l)['method'], json.loads(l)['top1'], json.loads(l)['loss_first20'], json.loads(l)['loss_last20']) for l in sys.stdin]"
grep -h '^{' gpurun_out/det_2.jsonl | python -c "import sys,json; [print(json.loads(l)['method'], json.loads(l)['top1'], json.loads(l)['loss_first20'], json.loads(l)['loss_last20']) for l in sys.stdin]"
