"""Per-step losses of the ResNet-9 convergence recipe (tests/test_convergence_gpu.py) for one
method / mode, to see where a run diverges."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from layer_wise_aaai20_amd.train.cifar_fast import CifarTrainer  # noqa: E402
from layer_wise_aaai20_amd.utils.logging import PiecewiseLinear  # noqa: E402

method, mode = sys.argv[1], sys.argv[2]
torch.manual_seed(0)
tr = CifarTrainer("resnet9", compress=mode, method=method, error_feedback=True, batch_size=128,
                  epochs=2, n_train=12800, seed=0, K=0.01,
                  graph=os.environ.get("PROBE_GRAPH", "1") == "1")
tr.steps_per_epoch = 1
if os.environ.get("PROBE_TORCH_AUG") == "1":
    tr.batches.use_kernel = False
tr.sched = PiecewiseLinear([0, 40, 200], [0, 0.4, 0])
ls = []
sync_each = os.environ.get("PROBE_SYNC") == "1"
keep = [] if os.environ.get("PROBE_KEEP") == "1" else None    # never free the batch tensors
for i in range(40):
    if sync_each:
        torch.cuda.synchronize()
    if keep is not None:
        b = tr.next_batch()
        if os.environ.get("PROBE_SYNC_AFTER_BATCH") == "1":
            torch.cuda.synchronize()
        if os.environ.get("PROBE_PRINT_STREAM") == "1" and i < 6:
            print("stream", torch.cuda.current_stream(), flush=True)
        keep.append(b)
        ls.append(float(tr.step(b)) / tr.bs)
    else:
        ls.append(float(tr.step()) / tr.bs)
print("graph", tr.graphed.enabled, "replays", tr.graphed.replays, "decided", tr.graphed.decided)
print(" ".join(f"{v:.2f}" for v in ls))
