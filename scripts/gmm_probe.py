import torch
a = torch.randn(512, 256, device="cuda", dtype=torch.bfloat16)
b = torch.randn(4, 256, 384, device="cuda", dtype=torch.bfloat16)
offs = torch.tensor([100, 256, 300, 512], device="cuda", dtype=torch.int32)
try:
    out = torch._grouped_mm(a, b, offs)
    ref = torch.cat([a[s:e].float() @ b[g].float() for g, (s, e) in enumerate(zip([0, 100, 256, 300], [100, 256, 300, 512]))])
    print("grouped_mm 2d3d ok", (out.float() - ref).abs().max().item())
    d = torch.randn(512, 384, device="cuda", dtype=torch.bfloat16)
    out2 = torch._grouped_mm(a.t(), d, offs)
    print("grouped_mm 2d2d ok", out2.shape)
except Exception as e:
    print("grouped_mm failed:", type(e).__name__, str(e)[:300])
