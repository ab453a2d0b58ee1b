import threading
import torch
from tony_amd.ops import _lib
from tony_amd.ops.pool import _box3

dev = torch.device("cuda", 0)
dy = torch.randn(4, 64, 35, 35, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
ref = torch.nn.functional.avg_pool2d(dy.float(), 3, 1, 1, count_include_pad=True)
print("main stream", _lib.stream_ptr(dev), torch.cuda.current_stream(dev))
out = _box3(dy, 4, 64, 35, 35, 64)
torch.cuda.synchronize()
print("main maxdiff", (out.float() - ref).abs().max().item())


class F(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        print("bwd thread", threading.current_thread().name, "stream", _lib.stream_ptr(g.device),
              torch.cuda.current_stream(g.device), "g strides", g.stride(), g.dtype, g.is_contiguous(memory_format=torch.channels_last))
        o = _box3(g, 4, 64, 35, 35, 64)
        torch.cuda.synchronize()
        r = torch.nn.functional.avg_pool2d(g.float(), 3, 1, 1, count_include_pad=True)
        print("bwd maxdiff", (o.float() - r).abs().max().item())
        o2 = _box3(g.contiguous(memory_format=torch.channels_last).clone(), 4, 64, 35, 35, 64)
        torch.cuda.synchronize()
        print("bwd maxdiff clone", (o2.float() - r).abs().max().item())
        return o


x = dy.clone().requires_grad_(True)
y = F.apply(x)
y.backward(dy)
