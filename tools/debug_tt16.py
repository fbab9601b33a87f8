import sys, torch, numpy as np
sys.path.insert(0, '/root/repo')
from fp8_quantization_amd import approx_calculation as ac
from fp8_quantization_amd.resnet_workload import resnet18_approx
DEV='cuda:0'
E,M=3,4
torch.manual_seed(E*10+M)
m = resnet18_approx(bn_stats_batches=2, device=DEV, expo_width=E, mant_width=M, withComp=False).to(DEV).eval()
g = torch.Generator().manual_seed(5)
m.quantized()
m.estimate_ranges()
conv0 = ac.approx_conv2d
n=[0]
saved=[]
def conv(xq, w, E_, M_, bA, bW, bR, table=None, **kw):
    y = conv0(xq, w, E_, M_, bA, bW, bR, table, **kw)
    n[0]+=1
    bad = torch.isnan(y).any().item() or torch.isinf(y).any().item()
    if bad and not saved:
        saved.append(1)
        nf = ~torch.isfinite(y)
        idx = nf.nonzero()
        print('nonfinite', int(nf.sum()), 'of', y.numel(), 'channels', sorted(set(idx[:, 1].tolist()))[:20], 'first', idx[:5].tolist())
        print('x absmax', xq.abs().max().item(), 'w absmax', w.abs().max().item(), 'y finite absmax', y[torch.isfinite(y)].abs().max().item())
        torch.save(dict(x=xq.cpu(), w=w.cpu(), bA=bA.cpu() if isinstance(bA, torch.Tensor) else bA, bW=bW.cpu() if isinstance(bW, torch.Tensor) else bW, bR=bR.cpu() if isinstance(bR, torch.Tensor) else bR), 'gpurun_out/bad_conv.pt')
    if bad or n[0] < 3:
        f = lambda t: t.reshape(-1)[:4].tolist() if isinstance(t, torch.Tensor) else t
        print('conv', n[0], 'shape', tuple(xq.shape), tuple(w.shape), 'bA', f(bA), 'bW', f(bW) if not isinstance(bW, torch.Tensor) else (bW.min().item(), bW.max().item()), 'bR', f(bR), 'nan/inf', bad, 'kw', {k: (v if not isinstance(v, torch.Tensor) else 'T') for k, v in kw.items()}, flush=True)
    return y
ac.approx_conv2d = conv
with torch.no_grad():
    out = m(torch.randn((4, 3, 64, 64), generator=g).to(DEV))
print('out nan', torch.isnan(out).any().item())

