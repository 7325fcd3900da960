#!/bin/bash
# Node preparation (reference IMAGENET/setup.sh fetched sorted_idxar.p, installed pillow-simd and
# tuned TCP sysctls for AWS). On an MI355X node: check the ROCm stack, GPUs and xGMI links, build
# the HIP extension in-tree, and optionally stage a dataset on local NVMe.
#   bash IMAGENET/setup.sh [--dataset SRC DST]
set -euo pipefail
cd "$(dirname "$0")/.."
echo "== ROCm"; ls -d /opt/rocm* 2>/dev/null || { echo "ROCm not found"; exit 1; }
command -v rocm-smi >/dev/null && rocm-smi --showproductname --showtopo 2>/dev/null | head -40 || true
echo "== PyTorch"
python - <<'PY'
import torch
print("torch", torch.__version__, "hip", torch.version.hip, "gpus", torch.cuda.device_count())
import torch.distributed as d
print("nccl(RCCL) backend", d.is_nccl_available(), "gloo", d.is_gloo_available())
PY
echo "== build HIP extension (gfx950)"
python -c "import __graft_entry__ as g; g.build()"
if [ "${1:-}" = "--dataset" ]; then
  python IMAGENET/tools/replicate_imagenet.py --src "$2" --dst "$3"
fi
echo "setup ok"
