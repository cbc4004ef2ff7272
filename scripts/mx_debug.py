import torch, sys
sys.path.insert(0, '/root/repo')
from lightning_thunder_amd.ops.fp8 import mx_quantize, mx_dequantize, gemm_nt_mx
torch.manual_seed(0)
M, N, K = 256, 256, 256
a = torch.randn(M, K, device="cuda").bfloat16()
b = torch.randn(N, K, device="cuda").bfloat16()
qa, sa, _, _ = mx_quantize(a)
qb, sb, _, _ = mx_quantize(b)
def check(tag, sa_, sb_):
    out = gemm_nt_mx(qa, sa_, qb, sb_, 0, 0).float()
    ref = mx_dequantize(qa, sa_) @ mx_dequantize(qb, sb_).t()
    print(tag, ((out - ref).norm() / ref.norm()).item(), flush=True)
    return out, ref
one_a = torch.full_like(sa, 127); one_b = torch.full_like(sb, 127)
check("unit", one_a, one_b)
check("real", sa, sb)
for blk in range(8):
    s2 = one_a.clone(); s2[:, blk] = 128
    check(f"a blk{blk}", s2, one_b)
for rows in (0, 16, 64, 128):
    s2 = one_a.clone(); s2[rows, :] = 128
    out, ref = check(f"a row{rows}", s2, one_b)
    d = (out - ref).abs().sum(1).nonzero().flatten().tolist()
    print("  bad rows", d[:10])
s2 = one_b.clone(); s2[:, 3] = 126
check("b blk3", one_a, s2)
