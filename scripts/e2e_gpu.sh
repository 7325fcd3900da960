#!/bin/bash
# End-to-end GPU run of the reference-compatible entry points on synthetic data: ImageNet
# train_imagenet_nv (2 short epochs with the smoke phase schedule, bf16, overlapped layer-wise Top-K
# + EF, checkpoint), resume from the checkpoint for one more epoch, evaluate-only; CIFAR dawn.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/e2e
OUT=gpurun_out/e2e
run() { local name=$1; shift; echo "=== $name"; timeout -k 10 300 "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -4 $OUT/$name.log; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run imagenet_train python IMAGENET/training/train_imagenet_nv.py synthetic --phases smoke --epochs 2 \
  --short-epoch --bf16 --overlap -c layerwise --method Topk -K 0.001 --error-feedback --init-bn0 \
  --no-bn-wd --logdir /tmp/e2e_run --extra-ckpt --print-freq 5
ls /tmp/e2e_run | tee $OUT/ckpt_files.txt
CK=$(ls /tmp/e2e_run/*.tar | head -1)
run imagenet_resume python IMAGENET/training/train_imagenet_nv.py synthetic --phases smoke --epochs 3 \
  --short-epoch --bf16 --overlap -c layerwise --method Topk -K 0.001 --error-feedback --init-bn0 \
  --no-bn-wd --logdir /tmp/e2e_run2 --resume "$CK" --print-freq 5
run imagenet_eval python IMAGENET/training/train_imagenet_nv.py synthetic --phases smoke --short-epoch \
  --bf16 --resume "$CK" --evaluate --logdir /tmp/e2e_run3
run cifar_dawn python -m CIFAR10.dawn -m tcp://127.0.0.1:29531 -r 0 -w 1 -n resnet9 -c layerwise \
  --method Topk -K 0.01 --epochs 1 --synthetic
echo e2e ok
