"""One-shot xGMI all-reduce kernel (csrc/hip/allreduce.hip) vs a torch sum.

The 1-GPU test box cannot run an 8-GPU job, so two processes share cuda:0:
they exchange hipIpc handles over a gloo group exactly as ranks on separate
GPUs do and run the same kernel (peer loads then go to local HBM instead of
over xGMI).  Covers several message sizes, both dtypes, repeated calls
(epoch/parity double buffering) and hipGraph capture + replay."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from ipex_llm_amd.parallel.comm import CustomAllReduce
        car = CustomAllReduce(None, device="cuda:0", max_bytes=1 << 21)
        for dt in (torch.bfloat16, torch.float16, torch.float32):
            for n in (8, 4096, 8 * 4096, 64 * 4096 + 8):
                if n * torch.finfo(dt).bits // 8 > car.cap:
                    continue
                for two in (0, 1):
                    for it in range(3):
                        g = torch.Generator(device="cuda").manual_seed(1000 * it + n)
                        base = torch.randn(world, n, generator=g, device="cuda").to(dt)
                        mine = base[rank].clone()
                        want = base.float().sum(0)
                        # in place (the decoder reduces its f32 accumulator where it lies)
                        out = car(mine, out=mine if it == 2 else None, two_shot=two)
                        err = ((out.float() - want).abs().max() / want.abs().max()).item()
                        tol = 1e-5 if dt == torch.float32 else 2e-2
                        assert err < tol, (dt, n, two, it, err)
        # graph capture: the epoch counters live on the device
        x = torch.full((4096,), float(rank + 1), device="cuda", dtype=torch.bfloat16)
        car(x)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            y = car(x)
        for v in range(3):
            x.fill_(float(rank + 1 + v))
            graph.replay()
            torch.cuda.synchronize()
            exp = sum(r + 1 + v for r in range(world))
            assert torch.all(y.float() == exp), (v, y[:4])
        car.check()
        car.close()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
        raise


@pytest.mark.parametrize("world", [2, 4])
def test_custom_all_reduce_procs_one_gpu(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(180)
    res = {}
    while not q.empty():
        r, m = q.get()
        res[r] = m
    for p in ps:
        if p.is_alive():
            p.kill()
    assert res == {r: "ok" for r in range(world)}, res


def _gather_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from ipex_llm_amd.parallel import comm
        car = comm.CustomAllReduce(None, device="cuda:0", max_bytes=1 << 20)
        for rows, n in ((1, 64), (8, 16032), (3, 8)):
            dt = torch.float32 if n == 8 else torch.bfloat16
            base = torch.arange(rows * n, device="cuda", dtype=torch.float32).view(rows, n)
            x = (base + 1e5 * rank).to(dt)
            want = torch.cat([(base + 1e5 * r).to(dt) for r in range(world)], -1)
            got = car.all_gather_last_dim(x)
            assert got.shape == (rows, world * n) and torch.equal(got.float(), want.float()), (rows, n)
        # interleaved with all-reduces (shared epochs) and captured
        x = torch.full((8, 256), float(rank), device="cuda", dtype=torch.bfloat16)
        car(x.clone())
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            y = car.all_gather_last_dim(x)
            z = car(x)
        for v in range(2):
            x.fill_(float(rank + v))
            graph.replay()
            torch.cuda.synchronize()
            assert all(torch.all(y[:, r * 256:(r + 1) * 256].float() == r + v) for r in range(world))
            assert torch.all(z.float() == sum(r + v for r in range(world)))
        car.check()
        car.close()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
        raise


def _missing_peer_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        import ipex_llm_amd.ops as ops
        from ipex_llm_amd.parallel.comm import CustomAllReduce
        car = CustomAllReduce(None, device="cuda:0", max_bytes=1 << 20)
        if rank == 0:                       # rank 1 never joins this call
            out = car(torch.ones(4096, device="cuda", dtype=torch.bfloat16))
            torch.cuda.synchronize()
            assert torch.isnan(out.float()).all(), out[:4]
            try:
                car.check()
                raise AssertionError("timeout not flagged")
            except RuntimeError as e:
                assert "timed out" in str(e)
            try:
                ops.check_kernel_errors()
                raise AssertionError("ERR_PEER not in the kernel error word")
            except ops.KernelError as e:
                assert "peer" in str(e)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
        raise


@pytest.mark.parametrize("fn", ["gather", "missing_peer"])
def test_custom_all_gather_and_missing_peer(fn):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    target = _gather_worker if fn == "gather" else _missing_peer_worker
    ps = [ctx.Process(target=target, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    res = {}
    while not q.empty():
        r, msg = q.get()
        res[r] = msg
    for p in ps:
        if p.is_alive():
            p.kill()
    assert res == {0: "ok", 1: "ok"}, res
