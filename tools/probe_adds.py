"""Which autograd ops launch elementwise bf16 adds in one 7B-dimension TransformerLayer fwd+bwd (GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.models import llama_architecture  # noqa: E402
from scaling_amd.transformer.context.config import TransformerArchitectureConfig  # noqa: E402
from scaling_amd.transformer.model.layers import TransformerLayer  # noqa: E402
from scaling_amd.transformer.model.layers.base import TransformerLayerIO  # noqa: E402

a = llama_architecture("llama2_7b", sequence_length=4096, precision="bfloat16", num_layers=1)
a["masked_softmax"] = {"kernel": "flash_attention"}
layer = TransformerLayer(TransformerArchitectureConfig.from_dict(a), layer_index=0).cuda()
S, B = 4096, 4
x = torch.randn(B, S, 4096, device="cuda", dtype=torch.bfloat16, requires_grad=True)
pos = torch.arange(S, device="cuda").repeat(B, 1)
cu = torch.arange(0, B * S + 1, S, device="cuda", dtype=torch.int32)


def run():
    io = TransformerLayerIO(activations=x, position_ids=pos, cumulative_seq_lengths=cu, cumulative_seq_lengths_padded=cu)
    y = layer(io).activations
    y.backward(torch.ones_like(y))


run()
torch.cuda.synchronize()
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
    run()
    torch.cuda.synchronize()
for e in prof.events():
    if e.name in ("aten::add", "aten::add_", "aten::fill_", "aten::zero_", "aten::copy_", "aten::cat"):
        st = [f for f in (e.stack or []) if "scaling_amd" in f][:4]
        print(e.name, e.input_shapes, st)
