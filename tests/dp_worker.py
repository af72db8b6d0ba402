"""Rank process for tests/test_dp_gpu.py (not collected by pytest).

    python tests/dp_worker.py single OUT
    python tests/dp_worker.py dp OUT RANK WORLD PORT [eager]

`dp`: one rank of a real process group (gloo; every rank on cuda:0, the 1-GPU
rehearsal of the one-process-per-GPU arrangement) running train.FastStTrainer on
its own contiguous shard of each global batch: one eager step, then two
train_step() calls (hipGraph capture + replay) -- the path static_train takes.
`single`: the same three global batches on one process, world 1.
Results are written with torch.save to OUT/<mode><rank>.pt.
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("STX_NO_LOGFILE", "1")

H = 64
GLOBAL_B = 4


def data():
    from styletransfer_amd import weights as W
    style = torch.from_numpy(W.synthetic_image(21, (1, 3, H, H)))
    batches = [torch.from_numpy(W.synthetic_image(700 + k, (GLOBAL_B, 3, H, H)))
               for k in range(3)]
    return style, batches


def main():
    mode, out = sys.argv[1], sys.argv[2]
    rank, world, graph, tag = 0, 1, True, mode
    if mode == "dp":
        rank, world, port = int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
        graph = not (len(sys.argv) > 6 and sys.argv[6] == "eager")
        tag = "dp" if graph else "dpeager"
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from styletransfer_amd import network
    from styletransfer_amd import weights as W
    from styletransfer_amd.train import FastStTrainer
    style, batches = data()
    style = style.to(dev)
    b = GLOBAL_B // world
    shards = [x[rank * b:(rank + 1) * b].to(dev).contiguous() for x in batches]
    net = network.ImageTransformNet(style, batch_size=b)
    # rank > 0 starts from different parameters: the trainer's broadcast must fix that
    net.load_state_dict({k: torch.from_numpy(v)
                         for k, v in W.itn_synthetic(4321 if rank == 0 else 999)})
    tr = FastStTrainer(net, style, world_size=world)
    res = {"p0": tr.flat.detach().cpu().clone()}
    with torch.no_grad():
        net(shards[0])  # primes the Conv2d weight-slab caches with the initial weights
    res["loss1"] = tr.step(shards[0]).detach().cpu().clone()
    res["grad1"] = tr.flat_grad.detach().cpu().clone()
    res["flat1"] = tr.flat.detach().cpu().clone()
    tr.train_step(shards[1], graph=graph)   # capture (its warm-up step trains on shard 1)
    tr.train_step(shards[2], graph=graph)   # replay
    torch.cuda.synchronize()
    res["flat3"] = tr.flat.detach().cpu().clone()
    # no-grad forward after training sees the updated weights (layers.Conv2d caches)
    with torch.no_grad():
        res["y_after"] = net(shards[0]).cpu()
        fresh = network.ImageTransformNet(style, batch_size=b)
        fresh.load_state_dict(net.state_dict())
        res["y_fresh"] = fresh(shards[0]).cpu()
    torch.save(res, os.path.join(out, f"{tag}{rank}.pt"))
    if mode == "dp":
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
