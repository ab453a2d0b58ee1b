import torch
from tony_amd.ops.pool import avg_pool3x3_s1
torch.manual_seed(0)
dev = torch.device("cuda", 0)
for fmt in [torch.contiguous_format, torch.channels_last]:
    for dt in [torch.float32, torch.bfloat16]:
        x = torch.randn(4, 64, 35, 35).to(dt).contiguous(memory_format=fmt)
        dy = torch.randn(4, 64, 35, 35).to(dt).contiguous(memory_format=fmt)
        xc = x.float().clone().requires_grad_(True)
        torch.nn.functional.avg_pool2d(xc, 3, 1, 1, count_include_pad=True).backward(dy.float())
        xg = x.to(dev).detach().requires_grad_(True)
        torch.nn.functional.avg_pool2d(xg, 3, 1, 1, count_include_pad=True).backward(dy.to(dev))
        print("torch gpu", fmt, dt, (xg.grad.float().cpu() - xc.grad).abs().max().item())
        if dt == torch.bfloat16 and fmt == torch.channels_last:
            xm = x.to(dev).detach().requires_grad_(True)
            avg_pool3x3_s1(xm).backward(dy.to(dev))
            print("tony gpu", (xm.grad.float().cpu() - xc.grad).abs().max().item())
