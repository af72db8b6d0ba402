"""Rank process for tests/test_dp_gpu.py::test_rccl_world1_exchange (not collected).

    python tests/rccl_worker.py OUT PORT

One rank with the torchrun environment (RANK 0, WORLD_SIZE 1) and an RCCL process
group (backend "nccl", device_id bound as bench.py does), running
train.FastStTrainer with that group: its step issues the flat-gradient SUM
all-reduce through RCCL even at world 1 (a process group forces the exchange), one
eager step and two train_step() calls (hipGraph capture with the all-reduce eager
between the two graphs, then a replay).  A group-less trainer on the same
parameters and batches runs in the same process; both parameter vectors and
whether librccl is mapped into the process are written to OUT/rccl.pt."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("STX_NO_LOGFILE", "1")


def main():
    out, port = sys.argv[1], sys.argv[2]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    pg = dist.group.WORLD
    from styletransfer_amd import network
    from styletransfer_amd import weights as W
    from styletransfer_amd.train import FastStTrainer
    H, B = 64, 2
    style = torch.from_numpy(W.synthetic_image(21, (1, 3, H, H))).to(dev)
    batches = [torch.from_numpy(W.synthetic_image(800 + k, (B, 3, H, H))).to(dev)
               for k in range(3)]
    res = {}
    for tag, group in (("rccl", pg), ("plain", None)):
        net = network.ImageTransformNet(style, batch_size=B)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)})
        tr = FastStTrainer(net, style, world_size=1, process_group=group)
        tr.step(batches[0])
        tr.train_step(batches[1])   # capture (its warm-up step trains on batch 1)
        tr.train_step(batches[2])   # replay: graph, eager RCCL all-reduce, graph
        torch.cuda.synchronize()
        res[f"{tag}_exchanges"] = tr.exchanges
        res[f"{tag}_flat"] = tr.flat.detach().cpu().clone()
        res[f"{tag}_grad"] = tr.flat_grad.detach().cpu().clone()
    with open("/proc/self/maps") as f:
        res["rccl_mapped"] = any("librccl" in ln for ln in f)
    res["backend"] = dist.get_backend(pg)
    torch.save(res, os.path.join(out, "rccl.pt"))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
