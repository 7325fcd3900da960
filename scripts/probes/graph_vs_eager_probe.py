"""Per-step parameter / EF / gradient comparison of the CIFAR trainer with and without the
HIP-graph step (argv: network mode method)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from layer_wise_aaai20_amd.train.cifar_fast import CifarTrainer  # noqa: E402

net, mode, method = sys.argv[1:4]
if "force" in sys.argv[4:]:                 # capture even the codecs kept eager (investigation)
    from layer_wise_aaai20_amd.compress import codecs as C
    C.RandkSparseCodec.graph_safe = True
runs = {}
ab = "overlap-ab" in sys.argv[4:]     # eager with the side stream vs eager inline instead
for graph in (False, True):
    if ab:
        os.environ["LWAAAI_OVERLAP"] = "0" if graph else "1"
    torch.manual_seed(0)
    tr = CifarTrainer(net, compress=mode, method=method, K=0.05, error_feedback=True,
                      batch_size=128, n_train=2560, graph=graph and not ab)
    hist = []
    for i in range(int(os.environ.get("PROBE_STEPS", "8"))):
        loss = float(tr.step())
        torch.cuda.synchronize()
        eng = tr.ddp.engine
        p = torch.cat([q.detach().float().reshape(-1) for q in tr.model.parameters()])
        hist.append((loss, p, eng.ef.clone(), eng.arena.grad.clone(), int(eng._dstep.item()),
                     eng.step))
    runs[graph] = hist
for i, (a, b) in enumerate(zip(runs[False], runs[True])):
    print(f"step {i}: loss {a[0]:.4f}/{b[0]:.4f}  dparam {float((a[1]-b[1]).abs().max()):.3e}  "
          f"def {float((a[2]-b[2]).abs().max()):.3e}  dgrad {float((a[3]-b[3]).abs().max()):.3e}  "
          f"nnz(grad) {int((a[3]!=0).sum())}/{int((b[3]!=0).sum())}  dstep {a[4]}/{b[4]} "
          f"host {a[5]}/{b[5]}", flush=True)
