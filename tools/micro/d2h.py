"""D2H probe: 256 MB (64 x 1M int32 labelings) device -> host, pageable fresh / pageable touched / pinned."""
import time
import numpy as np
import torch

n = 64 * 1000000
t = torch.arange(n, dtype=torch.int32, device="cuda:0")
torch.cuda.synchronize()
def tm(f, k=3):
    out = []
    for _ in range(k):
        torch.cuda.synchronize(); t0 = time.perf_counter(); f(); torch.cuda.synchronize(); out.append((time.perf_counter() - t0) * 1e3)
    return ["%.2f" % x for x in out]
print("fresh pageable t.cpu():", tm(lambda: t.cpu()))
dst = torch.empty(n, dtype=torch.int32); dst.fill_(1)
print("touched pageable copy_:", tm(lambda: dst.copy_(t)))
print("np.empty alloc+touch:", tm(lambda: np.empty(n, np.int32).fill(0)))
print("pinned alloc:", tm(lambda: torch.empty(n, dtype=torch.int32, pin_memory=True), 2))
pin = torch.empty(n, dtype=torch.int32, pin_memory=True)
print("pinned copy_:", tm(lambda: pin.copy_(t)))
a = np.empty(n, np.int32)
print("pinned->fresh np copy:", tm(lambda: np.copyto(np.empty(n, np.int32), pin.numpy())))

# hipMemcpyAsync kinds into a touched pageable numpy array (what labels_to_host does)
import ctypes
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
a = np.zeros(n, np.int32)
s = torch.cuda.current_stream().cuda_stream
for kind, name in ((2, "DeviceToHost"), (4, "Default")):
    def f():
        assert hip.hipMemcpyAsync(a.ctypes.data, t.data_ptr(), 4 * n, kind, s) == 0
        assert hip.hipStreamSynchronize(s) == 0
    print("hipMemcpyAsync %s touched pageable:" % name, tm(f))
