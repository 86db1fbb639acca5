import sys, os, json, torch
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "art-sbir_amd"))  # chunk-size sweep of knn_scan_v2 (1M x 512, 10k queries)
import _hip
dev = torch.device("cuda:0")
N, D, Q = 1_000_000, 512, 10_000
g = torch.randn(N, D, device=dev, generator=torch.Generator(device=dev).manual_seed(7))
pos = (torch.arange(Q, device=dev) * 7919) % N
q = g[pos] + 0.5 * torch.randn(Q, D, device=dev, generator=torch.Generator(device=dev).manual_seed(8))
L = _hip.lib(); s = torch.cuda.current_stream().cuda_stream
qsq = torch.empty(Q, device=dev); gsq = torch.empty(N, device=dev)
qc = torch.empty(Q, D, dtype=torch.bfloat16, device=dev); ga = torch.empty(N, D + 8, dtype=torch.bfloat16, device=dev)
_hip.call("artsbir_rows_prep", 1, q.data_ptr(), Q, D, qsq.data_ptr(), qc.data_ptr(), D, s)
_hip.call("artsbir_rows_prep_aug", g.data_ptr(), N, D, D, gsq.data_ptr(), ga.data_ptr(), s)
gmax = float(gsq.max())
for tpc in (128, 256, 512):
    nc = L.artsbir_knn_candidates_per_query(N, tpc)
    cd = torch.empty(Q, nc, device=dev); ci = torch.empty(Q, nc, dtype=torch.int32, device=dev)
    cnt = torch.zeros(Q, dtype=torch.int32, device=dev); unc = torch.zeros(2 * 4096 + 1, dtype=torch.int32, device=dev)
    ts = []
    for it in range(4):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        _hip.call("artsbir_knn_scan_aug", qc.data_ptr(), ga.data_ptr(), qsq.data_ptr(), gmax, Q, N, D, tpc, None, None, 0, 0.0,
                  None, None, cnt.data_ptr(), unc.data_ptr(), 4096, cd.data_ptr(), ci.data_ptr(), s)
        e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    print(json.dumps({"tpc": tpc, "ms": round(min(ts[1:]), 3)}), flush=True)
