import time, numpy as np, torch, threading
torch.cuda.set_device(0)
n = 120_000_000  # 480 MB of int32
a = np.arange(n, dtype=np.int32)
d = torch.empty(n, dtype=torch.int32, device='cuda')
torch.cuda.synchronize()
for rep in range(2):
    t=time.perf_counter(); d.copy_(torch.from_numpy(a)); torch.cuda.synchronize(); el=time.perf_counter()-t
    print('pageable H2D GB/s', round(a.nbytes/el/1e9,2))
p = torch.empty(n, dtype=torch.int32).pin_memory()
for rep in range(2):
    t=time.perf_counter(); p.numpy()[:] = a; el1=time.perf_counter()-t
    t=time.perf_counter(); d.copy_(p, non_blocking=True); torch.cuda.synchronize(); el2=time.perf_counter()-t
    print('memcpy->pinned GB/s', round(a.nbytes/el1/1e9,2), 'pinned H2D GB/s', round(a.nbytes/el2/1e9,2))
# threaded memcpy into pinned
pn = p.numpy()
def work(i, T):
    s = (n*i)//T; e=(n*(i+1))//T; pn[s:e] = a[s:e]
for T in (4, 8, 16):
    t=time.perf_counter(); th=[threading.Thread(target=work,args=(i,T)) for i in range(T)]
    [x.start() for x in th]; [x.join() for x in th]; el=time.perf_counter()-t
    print('threaded memcpy', T, 'GB/s', round(a.nbytes/el/1e9,2))
# D2H
for rep in range(2):
    t=time.perf_counter(); b=d.cpu(); el=time.perf_counter()-t
    print('D2H pageable GB/s', round(a.nbytes/el/1e9,2))
    t=time.perf_counter(); p.copy_(d); torch.cuda.synchronize(); el=time.perf_counter()-t
    print('D2H pinned GB/s', round(a.nbytes/el/1e9,2))
import ctypes
hip = ctypes.CDLL('libamdhip64.so')
for rep in range(2):
    t=time.perf_counter(); r=hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(a.nbytes), 0); el=time.perf_counter()-t
    print('hipHostRegister rc', r, 'GB/s', round(a.nbytes/el/1e9,2))
    t=time.perf_counter(); d.copy_(torch.from_numpy(a), non_blocking=True); torch.cuda.synchronize(); el2=time.perf_counter()-t
    print('registered H2D GB/s', round(a.nbytes/el2/1e9,2))
    t=time.perf_counter(); hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data)); print('unregister s', round(time.perf_counter()-t,4))
