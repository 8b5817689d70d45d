"""Native BEVNet head operand (model_wrapper.py:69-75: concat of the projected BEV map, the 2 positional channels and
the head's zero channel pad, channels-last) and its backward, bit-exact against the torch composition it replaces
(`(s + bias[:, None, None])` permuted to NHWC, cat with the positional map and zeros; the gradient's first P
channels back in NCHW).  Both kernel forms: the 16-B one (Wb % 4 == 0, cp % 4 == 0) and the scalar one (odd Wb or
cp), including ragged 64-cell runs at the row end and P not a multiple of 4.
"""
import pytest
import torch

import bev_native as nat

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def reference(s, bias, pos, cp):
    B, P, Hb, Wb = s.shape
    parts = [(s + bias[:, None, None]).permute(0, 2, 3, 1), pos.permute(1, 2, 0).unsqueeze(0).expand(B, Hb, Wb, 2)]
    if cp > P + 2:
        parts.append(s.new_zeros(B, Hb, Wb, cp - P - 2))
    return torch.cat(parts, dim=-1).contiguous()


@pytest.mark.parametrize("B,P,Hb,Wb,cp", [
    (1, 128, 24, 1440, 160),   # the BEV head geometry's row width and channel pad (16-B form)
    (2, 64, 7, 200, 68),       # 16-B form, ragged last run (200 = 3 x 64 + 8)
    (1, 128, 5, 101, 160),     # odd Wb -> scalar form
    (2, 30, 3, 70, 33),        # P % 4 != 0, odd cp -> scalar form
    (1, 62, 4, 96, 64),        # P % 4 != 0 in the 16-B form (the pos channels straddle a quad)
])
def test_head_operand_matches_torch(B, P, Hb, Wb, cp):
    g = torch.Generator(device="cpu").manual_seed(B * 1000 + P + Wb)
    s = torch.randn(B, P, Hb, Wb, generator=g).to(DEV)
    bias = torch.randn(P, generator=g).to(DEV)
    pos = torch.randn(2, Hb, Wb, generator=g).to(DEV)
    x = nat.head_operand(s, bias, pos, cp)
    torch.cuda.synchronize()
    assert torch.equal(x, reference(s, bias, pos, cp))
    gx = torch.randn(B, Hb, Wb, cp, generator=g).to(DEV)
    gs = nat.head_operand_bwd(gx, P)
    torch.cuda.synchronize()
    assert torch.equal(gs, gx[..., :P].permute(0, 3, 1, 2).contiguous())
    gs2, gb = nat.head_operand_bwd_bias(gx, P)  # with the bias gradient from the same pass (16-B form) or None
    torch.cuda.synchronize()
    assert torch.equal(gs2, gs)
    if Wb % 4 == 0 and cp % 4 == 0:
        ref = gx[..., :P].double().sum((0, 1, 2))
        assert gb is not None and gb.shape == (P,)
        # block partials in fp32 (64 cells each) added in double: within a few fp32 ulps of the exact sum
        assert float((gb.double() - ref).abs().max()) <= 1e-6 * float(gx[..., :P].abs().sum((0, 1, 2)).max())
    else:
        assert gb is None
