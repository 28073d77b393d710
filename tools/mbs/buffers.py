"""Same store kernel on a torch-allocated buffer vs a hipMalloc'd one, from one Python process."""
import ctypes
import os
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
torch.cuda.init()
lib = ctypes.CDLL(os.path.join(HERE, "libmbs.so"))
lib.mbs_store.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
lib.mbs_malloc.argtypes = [ctypes.c_size_t]
lib.mbs_malloc.restype = ctypes.c_void_p
n = 65536
nbytes = n * 297 * 4
tbuf = torch.empty(nbytes // 4, dtype=torch.int32, device="cuda")
raw = lib.mbs_malloc(nbytes + 4096)
s = torch.cuda.current_stream().cuda_stream


def t(ptr, reps=50):
    for _ in range(5):
        lib.mbs_store(ptr, n, s)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        lib.mbs_store(ptr, n, s)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / reps


for _ in range(2):
    print(f"torch buffer  {t(tbuf.data_ptr()):7.2f} us   hipMalloc buffer {t(raw):7.2f} us", flush=True)
io = torch.zeros(nbytes * 2 + 10 * n, dtype=torch.uint8, device="cuda")  # like Engine.io
print(f"torch io block {t(io.data_ptr()):7.2f} us", flush=True)
