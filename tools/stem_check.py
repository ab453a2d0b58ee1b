import torch, sys
sys.path.insert(0, '/root/repo')
from tony_amd.ops import conv as C
dev = torch.device('cuda', 0)
cl = torch.channels_last
for (n, h, co, k, s, p) in [(4, 64, 64, 7, 2, 3), (4, 64, 64, 7, 2, 3), (2, 224, 64, 7, 2, 3), (2, 299, 32, 3, 2, 0), (4, 64, 32, 3, 2, 1), (4, 64, 32, 3, 1, 1)]:
    torch.manual_seed(0)
    x = torch.randn(n, 3, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(co, 3, k, k, device=dev) / (3 * k * k) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    y = C.stem_fwd(x, w, s, p)
    ref = torch.nn.functional.conv2d(x.float(), w.float(), None, s, p)
    rel = ((y.float() - ref).norm() / ref.norm()).item()
    print(n, h, co, k, s, p, "rel", rel, flush=True)
