import time, torch, sys
sys.path.insert(0, ".")
from omldm_amd.ops import native
lib = native.hip()
dev = torch.device("cuda", 0)
n = 11 << 20
h = torch.empty(n, dtype=torch.uint8, pin_memory=True); h.fill_(1)
d = torch.empty(n, dtype=torch.uint8, device=dev)
def run(label, stream_handle, src_ptr, reps=10):
    enq = 0.0
    for r in range(reps + 2):
        t0 = time.perf_counter()
        rc = lib.omldm_h2d_async(d.data_ptr(), src_ptr, n, stream_handle)
        t1 = time.perf_counter()
        assert rc == 0
        torch.cuda.synchronize()
        if r >= 2: enq += t1 - t0
    t0 = time.perf_counter()
    for r in range(reps):
        lib.omldm_h2d_async(d.data_ptr(), src_ptr, n, stream_handle)
    torch.cuda.synchronize()
    tt = (time.perf_counter() - t0) / reps
    print(f"{label:40s} enqueue {enq/reps*1e6:8.1f} us   per copy {tt*1e6:8.1f} us  {n/tt/1e9:5.1f} GB/s", flush=True)
s_torch = torch.cuda.Stream(dev)
run("torch pinned, torch pool stream", s_torch.cuda_stream, h.data_ptr())
run("torch pinned, legacy default stream", 0, h.data_ptr())
raw = lib.omldm_stream_create_cumask(0)
run("torch pinned, native cumask(all) stream", raw, h.data_ptr())
# torch.Tensor.copy_
enq=0
for r in range(12):
    with torch.cuda.stream(s_torch):
        t0=time.perf_counter(); d.copy_(h, non_blocking=True); t1=time.perf_counter()
    torch.cuda.synchronize()
    if r>=2: enq+=t1-t0
print(f"{'torch copy_ non_blocking (pool stream)':40s} enqueue {enq/10*1e6:8.1f} us", flush=True)
# back-to-back copies: does the enqueue block while a previous copy is in flight?
torch.cuda.synchronize()
ts = []
for r in range(6):
    t0 = time.perf_counter()
    lib.omldm_h2d_async(d.data_ptr(), h.data_ptr(), n, s_torch.cuda_stream)
    ts.append((time.perf_counter() - t0) * 1e6)
torch.cuda.synchronize()
print("back-to-back same stream, enqueue us:", [round(x, 1) for x in ts], flush=True)
s2 = torch.cuda.Stream(dev)
d2 = torch.empty(n, dtype=torch.uint8, device=dev)
ts = []
for r in range(6):
    st = s_torch if r % 2 == 0 else s2
    dd = d if r % 2 == 0 else d2
    t0 = time.perf_counter()
    lib.omldm_h2d_async(dd.data_ptr(), h.data_ptr(), n, st.cuda_stream)
    ts.append((time.perf_counter() - t0) * 1e6)
torch.cuda.synchronize()
print("alternating two streams, enqueue us:", [round(x, 1) for x in ts], flush=True)
# copy while a kernel runs on the default stream
big = torch.randn(8192, 8192, device=dev)
torch.cuda.synchronize()
ts = []
for r in range(4):
    c = big @ big  # compute on the default stream
    t0 = time.perf_counter()
    lib.omldm_h2d_async(d.data_ptr(), h.data_ptr(), n, s_torch.cuda_stream)
    ts.append((time.perf_counter() - t0) * 1e6)
torch.cuda.synchronize()
print("copy enqueued while a GEMM runs, enqueue us:", [round(x, 1) for x in ts], flush=True)
# two halves of different slices (different src offsets)
ts = []
hs = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(3)]
for r in range(6):
    t0 = time.perf_counter()
    lib.omldm_h2d_async(d.data_ptr(), hs[r % 3].data_ptr(), n, s_torch.cuda_stream)
    ts.append((time.perf_counter() - t0) * 1e6)
torch.cuda.synchronize()
print("back-to-back, 3 different pinned sources, enqueue us:", [round(x, 1) for x in ts], flush=True)
# the bench's event pattern: copy k+1 on the copy stream ‖ compute k on the current stream
def pattern(label, use_consumed_wait, cur_stream=None):
    slots = 3
    dsts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(slots)]
    copied = [torch.cuda.Event() for _ in range(slots)]
    consumed = [torch.cuda.Event() for _ in range(slots)]
    cs = torch.cuda.Stream(dev)
    a = torch.randn(4096, 4096, device=dev)
    ctx = torch.cuda.stream(cur_stream) if cur_stream is not None else torch.cuda.stream(torch.cuda.current_stream())
    with ctx:
        for e in consumed:
            e.record()
        torch.cuda.synchronize()
        enq = []
        def prefetch(k):
            sl = k % slots
            with torch.cuda.stream(cs):
                if use_consumed_wait:
                    cs.wait_event(consumed[sl])
                t0 = time.perf_counter()
                lib.omldm_h2d_async(dsts[sl].data_ptr(), hs[k % 3].data_ptr(), n, cs.cuda_stream)
                enq.append((time.perf_counter() - t0) * 1e6)
                copied[sl].record(cs)
        prefetch(0)
        t_start = time.perf_counter()
        for k in range(20):
            prefetch(k + 1)
            sl = k % slots
            torch.cuda.current_stream().wait_event(copied[sl])
            c = a @ a
            consumed[sl].record()
        torch.cuda.synchronize()
        per = (time.perf_counter() - t_start) / 20 * 1e6
    print(f"{label:45s} step {per:7.1f} us  enqueue median {sorted(enq)[len(enq)//2]:7.1f} us max {max(enq):7.1f}", flush=True)
t0 = time.perf_counter(); c = torch.randn(4096, 4096, device=dev); torch.cuda.synchronize()
a = torch.randn(4096, 4096, device=dev); torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(10): c = a @ a
torch.cuda.synchronize(); print("GEMM alone us", (time.perf_counter() - t0) / 10 * 1e6)
pattern("pattern, consumed wait, default stream", True)
pattern("pattern, no consumed wait, default stream", False)
pattern("pattern, consumed wait, compute on pool stream", True, torch.cuda.Stream(dev))
pattern("pattern, no consumed wait, compute on pool stream", False, torch.cuda.Stream(dev))
