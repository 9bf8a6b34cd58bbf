import sys, time, torch
sys.path.insert(0, ".")
from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.synthetic import synth_batch
from omldm_amd.ops.serving import PredictServer
mode = sys.argv[1]
dev = torch.device("cuda", 0)
sp = FeatureSpace(13, 0, 26, 1 << 16, field_aware=True)
w = torch.randn(sp.dim, device=dev).to(torch.bfloat16)
if mode == "graph":
    x = torch.zeros(1024, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        x.add_(1)
    for _ in range(10): g.replay()
    torch.cuda.synchronize()
one = synth_batch(sp, 1, start=3, pin=True)
srv = PredictServer(w, sp.dn, sp.dc, True, sp.cat_span)
t = time.time(); srv.start(lifetime_us=5_000_000); print("start", time.time() - t)
try:
    for i in range(5):
        print(i, srv.request(one), srv.lib.omldm_serve_alive(srv.mb))
except TimeoutError as e:
    print("timeout", srv.lib.omldm_serve_alive(srv.mb))
srv.close()
