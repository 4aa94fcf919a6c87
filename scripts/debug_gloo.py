"""GPU-box debugging aid: tests/test_gpu_sharded.py's two-process gloo run
with progress prints and a traceback dump if a rank stalls."""
import faulthandler
import os
import sys

sys.path.insert(0, ".")


def main(rank, world, port):
    f = open("gpurun_out/gloo_rank%d.log" % rank, "w", buffering=1)
    faulthandler.dump_traceback_later(60, exit=True, file=f)
    import torch
    import torch.distributed as tdist
    from opentsdb_amd import dist as odist
    from opentsdb_amd.engine import Engine
    from tests import datasets
    from tests.test_gpu_sharded import QUERIES, _spec
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    print("init", file=f)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    e = Engine(0)
    hb = datasets.random_batch(205, n_series=50, n_groups=3, nan_frac=0.02)
    for agg, ds, fill in QUERIES:
        print("query", agg, ds, fill, file=f)
        spec = _spec(agg, ds, fill)
        db = odist.to_device(odist.shard_host_batch(hb, world, rank))
        odist.run_sharded_any(e, spec, db, hb.n_groups)
        torch.cuda.synchronize()
        print("  done", file=f)
    tdist.barrier()
    print("end", file=f)


if __name__ == "__main__":
    import torch.multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=main, args=(r, 2, port)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=150)
        print("exit", p.exitcode)
