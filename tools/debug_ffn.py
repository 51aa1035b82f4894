import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch import nn
from bm2f_amd import linear_ops as lo

def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm()).item()

dev = torch.device("cuda")
torch.manual_seed(5)
l1, l2 = nn.Linear(256, 1024).to(dev), nn.Linear(1024, 256).to(dev)
x = torch.randn(3333, 256, device=dev)
g = torch.randn(3333, 256, device=dev)
h = lo.gemm_nt(x, l1.weight, l1.bias, relu=True)
href = torch.relu(x.double() @ l1.weight.double().t() + l1.bias.double())
print("h", rel(h, href), "zeros", (h == 0).float().mean().item(), "mismatch zero", ((h == 0) != (href == 0)).sum().item())
gh = lo.gemm_nt(g, l2.weight.t().contiguous(), mask=h)
ghref = torch.where(href > 0, g.double() @ l2.weight.double(), torch.zeros((), dtype=torch.float64, device=dev))
print("gh", rel(gh, ghref))
gh2 = torch.where(h > 0, g @ l2.weight, torch.zeros((), device=dev))
print("gh vs torch-where", rel(gh, gh2))
dw1, db1 = lo.gemm_tn(gh, x, colsum=True)
print("dw1 (from our gh)", rel(dw1, gh.double().t() @ x.double()), "db1", rel(db1, gh.double().sum(0)))
print("dw1 vs full ref", rel(dw1, ghref.t() @ x.double()))
for M in (3333, 3456, 3300, 3200, 10000):
    a = torch.randn(M, 1024, device=dev); b = torch.randn(M, 256, device=dev)
    c, cs = lo.gemm_tn(a, b, colsum=True)
    print("tn", M, rel(c, a.double().t() @ b.double()), rel(cs, a.double().sum(0)))
    a[:, ::3] = 0
    c, cs = lo.gemm_tn(a, b, colsum=True)
    print("tn sparse", M, rel(c, a.double().t() @ b.double()), rel(cs, a.double().sum(0)))
