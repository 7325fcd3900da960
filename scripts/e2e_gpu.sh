#!/bin/bash
# End-to-end GPU run of the reference-compatible entry points on synthetic data:
#  * ImageNet train_imagenet_nv (fast path: fused MFMA ResNet-50, CompressedDDP, FlatSGD) at the
#    bench shape (bs 256, 224 px) — its logged step time is compared with bench.py;
#  * 2 short epochs with layer-wise Top-K + EF and --extra-ckpt, resume (EF residuals restored),
#    evaluate-only;
#  * CIFAR dawn (ResNet-9 and VGG-16, fast path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/e2e
OUT=gpurun_out/e2e
run() { local name=$1; shift; echo "=== $name"; timeout -k 10 400 "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -4 $OUT/$name.log; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
PH="[{'ep':0,'sz':224,'bs':256},{'ep':(0,1),'lr':(0.1,0.2)}]"
run imagenet_speed python IMAGENET/training/train_imagenet_nv.py synthetic --phases "$PH" \
  --epochs 1 --synthetic-size 10240 -c layerwise --method Topk -K 0.001 --init-bn0 --no-bn-wd \
  --logdir /tmp/e2e_speed --print-freq 10
grep -E "Epoch: \[0\]\[(20|30|40)/" /tmp/e2e_speed/verbose.log > $OUT/speed_lines.txt || true
cat $OUT/speed_lines.txt
run bench python bench.py --steps 20 --warmup 8
run imagenet_train python IMAGENET/training/train_imagenet_nv.py synthetic --phases smoke --epochs 2 \
  --short-epoch --bf16 -c layerwise --method Topk -K 0.001 --error-feedback --init-bn0 \
  --no-bn-wd --logdir /tmp/e2e_run --extra-ckpt --print-freq 5
ls /tmp/e2e_run | tee $OUT/ckpt_files.txt
CK=/tmp/e2e_run/checkpoint.pth.tar
run imagenet_resume python IMAGENET/training/train_imagenet_nv.py synthetic --phases smoke --epochs 3 \
  --short-epoch --bf16 -c layerwise --method Topk -K 0.001 --error-feedback --init-bn0 \
  --no-bn-wd --logdir /tmp/e2e_run2 --resume "$CK" --print-freq 5
grep -h "EF residual" $OUT/imagenet_train.log $OUT/imagenet_resume.log | tee $OUT/ef_check.txt
run imagenet_eval python IMAGENET/training/train_imagenet_nv.py synthetic --phases smoke --short-epoch \
  --bf16 --resume "$CK" --evaluate --logdir /tmp/e2e_run3
run cifar_resnet9 python -m CIFAR10.dawn -m tcp://127.0.0.1:29531 -r 0 -w 1 -n resnet9 -c layerwise \
  --method Topk -K 0.01 --epochs 1 --synthetic
run cifar_vgg16 python -m CIFAR10.dawn -m tcp://127.0.0.1:29532 -r 0 -w 1 -n vgg16 -c layerwise \
  --method Topk -K 0.001 --epochs 1 --synthetic --n_train 10240
echo e2e ok
