import torch, sys
sys.path.insert(0, '.')
from tony_amd.models.inception_v3 import inception_v3
from tony_amd.models.layers import cast_model
from tony_amd.ops import tape
cuda = torch.device('cuda', 0)
m = cast_model(inception_v3(num_classes=100, fused=True, seed=3), torch.bfloat16, cuda).to(memory_format=torch.channels_last).train()
m.dropout.p = 0.0
x = torch.randn(32, 3, 299, 299, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for use in (False, True):
    tape.ENABLED = use
    m.zero_grad(set_to_none=True)
    logits, aux = m(x)
    (logits.float().sum() + aux.float().sum()).backward()
    torch.cuda.synchronize()
    missing = [n for n, p in m.named_parameters() if p.grad is None]
    print("tape", use, "missing", len(missing), missing)
