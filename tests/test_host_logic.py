"""Host-side logic of the drop-in modules (CPU only, no kernel launches).

Calibration conventions (geometry.py:96-118, 33-64), module surface and
state_dict names, encoder input checks (cnn_encoder.py:50-72), fusion mode
assertion (fusion.py:14), ConcatFusion (fusion.py:39-46).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN


def test_gather_calibration_matches_reference_homography_rules():
    from models.fusion.geometry import gather_calibration
    d = np.load(os.path.join(GOLDEN, "homography_cases.npz"))
    for k in sorted({f.rsplit("_", 1)[0] for f in d.files}):
        K = torch.from_numpy(d[k + "_K"])
        Rt = torch.from_numpy(d[k + "_Rt"])
        # a single matrix is broadcast to every (b, v) by the reference's get_K/get_Rt
        if K.dim() == 2 and Rt.dim() == 2:
            K33, G33 = gather_calibration(K, Rt, 1, 1, torch.device("cpu"))
        else:  # 1-D Rt: per-view list form goes through _compute_homography's identity branch
            K33, G33 = gather_calibration([[K]], [[Rt]], 1, 1, torch.device("cpu"))
        H = (K33[0] @ G33[0]).numpy()  # same torch CPU matmul the reference uses (geometry.py:63)
        assert np.array_equal(H.view(np.uint32), d[k + "_H"].view(np.uint32)), k


def test_gather_calibration_tensor_and_list_forms_agree():
    from models.fusion.geometry import gather_calibration
    import bev_rig
    K, Rt = bev_rig.rig(3, 270, 480, 2)
    Kt, Rtt = torch.from_numpy(K), torch.from_numpy(Rt)
    a = gather_calibration(Kt, Rtt, 2, 3, torch.device("cpu"))
    b = gather_calibration([[Kt[i, j] for j in range(3)] for i in range(2)],
                           [[Rtt[i, j] for j in range(3)] for i in range(2)], 2, 3, torch.device("cpu"))
    c = gather_calibration(Kt[0], Rtt[0], 2, 3, torch.device("cpu"))  # [V,...] broadcast over frames
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert torch.equal(c[0][:3], a[0][:3]) and torch.equal(c[0][3:], a[0][:3])
    assert a[0].shape == (6, 3, 3) and a[1].shape == (6, 3, 3)


def test_geometry_module_surface():
    from models.fusion.geometry import GeometryTransformer, ViewProjection
    d = np.load(os.path.join(GOLDEN, "warp_w4_odd.npz"))
    g = GeometryTransformer(97, 301, (-24.0, 24.0, -7.2, 7.2), warp_impl="kornia")
    assert ViewProjection is GeometryTransformer
    assert g.warp_impl == "kornia" and GeometryTransformer(2, 2, (0, 1, 0, 1), "bogus").warp_impl == "grid_sample"
    assert tuple(g.ground_grid.shape) == (97, 301, 3)
    assert np.array_equal(g.ground_grid[0, :, 0].numpy().view(np.uint32), d["xs"].view(np.uint32))
    assert np.array_equal(g.ground_grid[:, 0, 1].numpy().view(np.uint32), d["ys"].view(np.uint32))
    assert "ground_grid" not in g.state_dict()  # non-persistent buffer (geometry.py:21)
    assert g.res_x == 48.0 / 301 and g.res_y == 14.4 / 97
    H = GeometryTransformer._compute_homography(torch.eye(3), torch.eye(4))
    assert torch.equal(H, torch.diag(torch.tensor([1.0, 1.0, 0.0])))  # [r1 r2 t] with t = 0
    Rt = torch.eye(4)
    Rt[2, 3] = 5.0
    Hi = GeometryTransformer._compute_img_to_world_homography(torch.eye(3) * 2, Rt)
    Hw = torch.diag(torch.tensor([2.0, 2.0, 10.0]))
    assert torch.allclose(Hi, torch.linalg.inv(Hw))
    Hs = GeometryTransformer._compute_img_to_world_homography(torch.eye(3), torch.eye(4))  # singular -> pinv
    assert torch.allclose(Hs, torch.linalg.pinv(torch.diag(torch.tensor([1.0, 1.0, 0.0]))))


def test_cpu_tensors_are_rejected_no_fallback():
    from models.fusion.geometry import GeometryTransformer
    g = GeometryTransformer(4, 6, (-1.0, 1.0, -1.0, 1.0))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        g(torch.zeros(1, 2, 3, 5, 5), torch.eye(3).expand(1, 2, 3, 3), torch.eye(4).expand(1, 2, 4, 4))


def test_fusion_module_surface():
    from models.fusion.fusion import SimpleFusion, ConcatFusion, AttentionFusion, FusionModule, BEVFusion
    with pytest.raises(AssertionError):
        SimpleFusion("avg")
    assert BEVFusion is SimpleFusion and SimpleFusion().mode == "sum"
    x = torch.randn(2, 3, 4, 5, 6)
    assert torch.equal(ConcatFusion()(x), x.reshape(2, 12, 5, 6))
    with pytest.raises(NotImplementedError):
        FusionModule()(x)
    assert isinstance(AttentionFusion(), FusionModule)


def test_encoder_surface_and_state_dict_names():
    from models.encoders.cnn_encoder import CNNEncoder, Backbone
    assert Backbone is CNNEncoder
    e = CNNEncoder(out_channels=64, backbone="resnet50", pretrained=False)
    keys = set(e.state_dict())
    for k in ("backbone.conv1.weight", "backbone.bn1.running_var", "backbone.layer1.0.downsample.0.weight",
              "backbone.layer2.3.conv3.weight", "backbone.layer4.2.bn3.bias"):
        assert k in keys, k
    assert not any(k.startswith("proj.") for k in keys)  # lazy proj (cnn_encoder.py:43-46)
    assert e._use_timm and e.out_index == 2
    f = CNNEncoder(out_channels=8, backbone="not_a_net", pretrained=False)
    assert not f._use_timm
    assert set(f.state_dict()) == {"backbone.0.weight", "backbone.0.bias", "backbone.2.weight", "backbone.2.bias"}
    with pytest.raises(ValueError):
        e(torch.zeros(3, 32, 32))
    with pytest.raises(ValueError):
        CNNEncoder(backbone_impl="gpu")


def test_img_to_world_homography_matches_reference_fixture():
    """GeometryTransformer._compute_img_to_world_homography (geometry.py:66-78) vs the reference's own outputs
    (tests/golden/img2world_cases.npz): Appendix-B rig, random calibrations, exactly singular and |det| < 1e-8
    (pinv branch).  Inverse via LAPACK on both sides: rel 1e-5 of each matrix's scale."""
    import numpy as np
    from models.fusion.geometry import GeometryTransformer
    d = np.load(os.path.join(GOLDEN, "img2world_cases.npz"))
    for K, Rt, ref in zip(d["K"], d["Rt"], d["H_i2w"]):
        got = GeometryTransformer._compute_img_to_world_homography(torch.from_numpy(K), torch.from_numpy(Rt)).numpy()
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-5 * max(np.abs(ref).max(), 1e-12))
