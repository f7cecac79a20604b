"""Two processes on cuda:0: rank 1 writes into rank 0's IPC-exported buffer by several copy
kinds; rank 0 reports what landed.  usage: python scripts/ipc_probe.py"""
import ctypes
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, port, q):
    import torch
    import torch.distributed as dist
    from merpcr_amd import _native
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    torch.cuda.set_device(0)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    pad = torch.zeros(100000, dtype=torch.uint8, device="cuda:0")  # buf at an offset inside its block
    buf = torch.zeros(4 * 1024, dtype=torch.uint8, device="cuda:0") if rank == 0 else None
    obj = [_native.ipc_handle(buf.data_ptr()) if rank == 0 else None]  # (handle, offset)
    dist.broadcast_object_list(obj, src=0)
    res = {}
    if rank == 1:
        p = _native.ipc_open(obj[0][0], 0) + obj[0][1]
        src = torch.arange(4 * 1024, dtype=torch.int32, device="cuda:0").to(torch.uint8)
        hsrc = torch.full((1024,), 7, dtype=torch.uint8).pin_memory()
        st = torch.cuda.Stream()
        res["nocu"] = hip.hipMemcpyAsync(p, src.data_ptr(), 1024, 1024, st.cuda_stream)        # D2D NoCU
        res["d2d"] = hip.hipMemcpyAsync(p + 1024, src.data_ptr() + 1024, 1024, 3, st.cuda_stream)  # D2D
        res["h2d"] = hip.hipMemcpyAsync(p + 2048, hsrc.data_ptr(), 1024, 1, st.cuda_stream)    # H2D pinned
        res["sync"] = hip.hipMemcpy(p + 3072, src.data_ptr() + 3072, 1024, 3)
        st.synchronize()
        torch.cuda.synchronize()
    dist.barrier()
    if rank == 0:
        b = buf.cpu()
        q.put({"nocu": int((b[:1024] != 0).sum()), "d2d": int((b[1024:2048] != 0).sum()),
               "h2d": int((b[2048:3072] == 7).sum()), "sync": int((b[3072:] != 0).sum())})
    else:
        q.put({"rc": res, "offset": obj[0][1]})
    dist.barrier()
    if rank == 1:
        _native.ipc_close(p - obj[0][1])
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as tmp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120), q.get(timeout=120)]
    for p in ps:
        p.join(timeout=60)
    print("landed bytes (of 1024 each) / rank-1 return codes and offset:", out, [p.exitcode for p in ps])
