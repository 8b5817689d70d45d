"""Wildtrack data path (reference project/data/wildtrack_loader.py, transforms.py).

The reference helpers themselves are pinned bit for bit by tests/test_wildtrack_golden.py (fixtures recorded
from the reference module with a raising torchvision stub for its unused module-scope import).  This file adds
known answers built from the dataset's published file formats:
OpenCV-storage intrinsics (`camera_matrix` with a `<data>` child) and Rodrigues extrinsics
(`rvec` / `tvec` in centimetres -> the reference's >100 "millimetre" rule divides by 1000), and the
Wildtrack annotation list (per-view boxes, bottom centre projected through inv(K [r1 r2 t])).
Expected values are computed independently (numpy / scipy in float64) and, for the world centres,
by the reference's own per-point float32 recipe restated inline (`_ref_pixel_to_world`).
The GPU tests pin the on-device ToTensor + Normalize kernel bit-exact and run a dataset batch
through BEVNet.
"""
import json
import math
import os

import numpy as np
import pytest
import torch
from PIL import Image

from data import transforms as T
from data.wildtrack_loader import (WildtrackDataset, _discover_camera_xmls, _load_camera_xml,
                                   _load_wildtrack_calibrations, _parse_float_list, _pixel_to_world, _rodrigues,
                                   _try_get_matrix, collate_fn)

CAMS = ["CVLab1", "CVLab2", "CVLab3", "CVLab4", "IDIAP1", "IDIAP2", "IDIAP3"]
IMG_HW = (54, 96)  # tiny frames; calibration at 1080 x 1920 as in Wildtrack


def _rig(v):
    """A Wildtrack-like camera v: K at 1080p, rvec (rad), tvec (cm)."""
    K = np.array([[1700.0 + 20 * v, 0.0, 960.0 - 5 * v], [0.0, 1690.0 + 10 * v, 540.0 + 3 * v], [0.0, 0.0, 1.0]])
    rvec = np.array([1.7 + 0.05 * v, 0.4 - 0.1 * v, -0.3 + 0.07 * v])
    tvec = np.array([-500.0 + 80 * v, 45.0 - 10 * v, 990.0 + 15 * v])
    return K, rvec, tvec


def _write_intrinsic(path, K):
    data = " ".join(f"{x:.10e}" for x in K.reshape(-1))
    path.write_text('<?xml version="1.0"?>\n<opencv_storage>\n<camera_matrix type_id="opencv-matrix">\n'
                    f"  <rows>3</rows>\n  <cols>3</cols>\n  <dt>d</dt>\n  <data>\n    {data}</data></camera_matrix>\n"
                    '<distortion_coefficients type_id="opencv-matrix">\n  <rows>5</rows>\n  <cols>1</cols>\n'
                    "  <dt>d</dt>\n  <data>\n    -0.3 0.1 0. 0. 0.</data></distortion_coefficients>\n"
                    "</opencv_storage>\n")


def _write_extrinsic(path, rvec, tvec):
    path.write_text('<?xml version="1.0"?>\n<opencv_storage>\n'
                    f"<rvec>{' '.join(repr(float(x)) for x in rvec)}</rvec>\n"
                    f"<tvec>{' '.join(repr(float(x)) for x in tvec)}</tvec>\n</opencv_storage>\n")


def _people():
    return [
        {"personID": 0, "positionID": 11, "views": [
            {"viewNum": 0, "xmin": 100, "ymin": 300, "xmax": 160, "ymax": 620},
            {"viewNum": 3, "xmin": 880, "ymin": 200, "xmax": 950, "ymax": 530},
            {"viewNum": 6, "xmin": 1200, "ymin": 400, "xmax": 1290, "ymax": 800}]},
        {"personID": 1, "positionID": 12, "views": [
            {"viewNum": 2, "xmin": 500, "ymin": 100, "xmax": 540, "ymax": 333},
            {"viewNum": 9, "xmin": 1, "ymin": 1, "xmax": 2, "ymax": 2},  # camera index out of range: skipped
            {"viewNum": 4, "xmin": None, "ymin": 1, "xmax": 2, "ymax": 2}]},  # incomplete box: skipped
        {"personID": 2, "positionID": 13, "views": [{"viewNum": 1, "xmin": 10, "ymin": 10}]},  # no ground point
    ]


@pytest.fixture(scope="module")
def wildtrack_root(tmp_path_factory):
    root = tmp_path_factory.mktemp("Wildtrack")
    (root / "calibrations" / "intrinsic_zero").mkdir(parents=True)
    (root / "calibrations" / "extrinsic").mkdir(parents=True)
    # the reference looks for Calibration / Calibrations / calibration
    os.rename(root / "calibrations", root / "calibration")
    for v, name in enumerate(CAMS):
        K, rvec, tvec = _rig(v)
        _write_intrinsic(root / "calibration" / "intrinsic_zero" / f"intr_{name}.xml", K)
        _write_extrinsic(root / "calibration" / "extrinsic" / f"extr_{name}.xml", rvec, tvec)
    rng = np.random.default_rng(0)
    for i in range(1, 8):
        d = root / "Image_subsets" / f"C{i}"
        d.mkdir(parents=True)
        for f in range(3):
            arr = rng.integers(0, 256, size=(108, 192, 3), dtype=np.uint8)
            Image.fromarray(arr).save(d / f"{5 * f:08d}.png")
    ann = root / "annotations_positions"
    ann.mkdir()
    (ann / "00000000.json").write_text(json.dumps(_people()))
    (ann / "00000005.json").write_text(json.dumps({"annotations": [{"world_pos": [1.5, -2.0]},
                                                                   {"world_pos": [3.0]}]}))
    (ann / "00000010.json").write_text("{ not json")
    return root


def _cfg(root, views=7):
    return {"DATA": {"DATA_ROOT": str(root), "VIEWS": views, "IMG_SIZE": [3, IMG_HW[0], IMG_HW[1]], "BATCH_SIZE": 2},
            "LOSS": {"DEFAULT_BOX_WH": [0.5, 0.7]}}


def _ref_pixel_to_world(u, v, K, Rt):
    """The reference's per-point recipe (wildtrack_loader.py:18-44), restated in torch float32."""
    G = torch.eye(3, dtype=torch.float32)
    G[:, :2] = Rt[:3, :2]
    G[:, 2:3] = Rt[:3, 3:4]
    Hi = torch.linalg.inv(K @ G)
    xyw = Hi @ torch.tensor([u, v, 1.0], dtype=torch.float32).reshape(3, 1)
    w = float(xyw[2, 0])
    if not (w == w) or abs(w) < 1e-8:
        return None
    return float(xyw[0, 0] / w), float(xyw[1, 0] / w)


def test_parse_float_list_and_matrix_tags():
    assert _parse_float_list("1, 2;3\n4\t5  six 7e-1") == [1.0, 2.0, 3.0, 4.0, 5.0, 0.7]
    assert _parse_float_list(None) == []
    import xml.etree.ElementTree as ET
    root = ET.fromstring("<r><A><x>1</x><x>2</x><x>3</x><x>4 5 6</x><x>7 8 9</x></A><T>1 2 3</T></r>")
    assert torch.equal(_try_get_matrix(root, ["K", "A"], (3, 3)), torch.arange(1, 10, dtype=torch.float32).view(3, 3))
    assert torch.equal(_try_get_matrix(root, ["T"], (3, 1)), torch.tensor([[1.0], [2.0], [3.0]]))
    assert _try_get_matrix(root, ["T"], (3, 3)) is None


def test_load_camera_xml_variants(tmp_path):
    p = tmp_path / "cam-C2.xml"  # the token must stand alone: "cam_C2" does not match (\w before C)
    p.write_text("<c><K>2 0 3 0 4 5 0 0 1</K><RT>1 0 0 10 0 1 0 20 0 0 1 30</RT></c>")
    K, Rt = _load_camera_xml(p)
    assert torch.equal(K, torch.tensor([[2.0, 0, 3], [0, 4, 5], [0, 0, 1]]))
    assert torch.equal(Rt[:3, 3], torch.tensor([10.0, 20.0, 30.0])) and torch.equal(Rt[3], torch.tensor([0.0, 0, 0, 1]))
    q = tmp_path / "x-3.xml"
    q.write_text("<c><rotation>0 -1 0 1 0 0 0 0 1</rotation><translation>1;2;3</translation></c>")
    K2, Rt2 = _load_camera_xml(q)
    assert torch.equal(K2, torch.diag(torch.tensor([1000.0, 1000.0, 1.0])))  # default K
    assert torch.equal(Rt2[:3, :3], torch.tensor([[0.0, -1, 0], [1, 0, 0], [0, 0, 1]]))
    empty = tmp_path / "none.xml"
    empty.write_text("<c/>")
    assert torch.equal(_load_camera_xml(empty)[1], torch.eye(4))
    found = _discover_camera_xmls(tmp_path, 4)
    assert found[1] == p and found[2] == q and found[0] is None and found[3] is None


def test_rodrigues_matches_rotvec():
    from scipy.spatial.transform import Rotation
    for v in range(7):
        _, rvec, _ = _rig(v)
        R = _rodrigues(torch.tensor(rvec, dtype=torch.float32).view(3, 1)).double().numpy()
        ref = Rotation.from_rotvec(rvec.astype(np.float32).astype(np.float64)).as_matrix()
        assert np.abs(R - ref).max() < 2e-6
    assert torch.equal(_rodrigues(torch.zeros(3)), torch.eye(3))


def test_wildtrack_calibrations(wildtrack_root):
    Ks, Rts = _load_wildtrack_calibrations(wildtrack_root / "calibration", 7)
    from scipy.spatial.transform import Rotation
    for v in range(7):
        K, rvec, tvec = _rig(v)
        assert np.array_equal(Ks[v].numpy(), K.astype(np.float32))
        R = Rotation.from_rotvec(rvec.astype(np.float32).astype(np.float64)).as_matrix()
        assert np.abs(Rts[v][:3, :3].double().numpy() - R).max() < 2e-6
        # |tvec| > 100 -> treated as millimetres: float32 tvec / 1000
        assert np.array_equal(Rts[v][:3, 3].numpy(), tvec.astype(np.float32) / np.float32(1000.0))
        assert torch.equal(Rts[v][3], torch.tensor([0.0, 0, 0, 1]))


def test_calibration_defaults_and_non7_naming(tmp_path, capsys):
    (tmp_path / "extrinsic").mkdir()
    _write_extrinsic(tmp_path / "extrinsic" / "extr_IDIAP2.xml", np.zeros(3), np.array([1.0, 2.0, 3.0]))
    _write_intrinsic(tmp_path / "intr_CVLab3.xml", np.diag([5.0, 6.0, 1.0]))
    Ks, Rts = _load_wildtrack_calibrations(tmp_path, 3)  # names: CVLab3, IDIAP2, then Cam3
    assert np.array_equal(Ks[0].numpy(), np.diag([5.0, 6.0, 1.0]).astype(np.float32))
    assert torch.equal(Ks[1], torch.diag(torch.tensor([1000.0, 1000.0, 1.0])))
    assert torch.equal(Rts[0], torch.eye(4))  # no extrinsic for CVLab3
    assert torch.equal(Rts[1][:3, 3], torch.tensor([1.0, 2.0, 3.0]))  # small norm: kept in metres
    assert "warning" in capsys.readouterr().out


def test_dataset_targets(wildtrack_root):
    ds = WildtrackDataset(_cfg(wildtrack_root))
    assert len(ds) == 3 and ds.frame_files == ["00000000.png", "00000005.png", "00000010.png"]
    Ks, Rts = ds.intrinsics[0], ds.extrinsics[0]
    t0 = ds.targets_per_frame[0]
    # person 0: mean over 3 views; person 1: one valid view; person 2: no ground point -> absent
    want = []
    for person in _people():
        pts = []
        for view in person["views"]:
            v = view["viewNum"]
            box = [view.get(k) for k in ("xmin", "xmax", "ymin", "ymax")]
            if v >= 7 or None in box:
                continue
            wp = _ref_pixel_to_world(0.5 * (box[0] + box[1]), float(box[3]), Ks[v], Rts[v])
            if wp is not None:
                pts.append(wp)
        if pts:
            want.append([sum(p[0] for p in pts) / len(pts), sum(p[1] for p in pts) / len(pts)])
    assert t0["centers_world"].shape == (2, 2)
    np.testing.assert_allclose(t0["centers_world"].numpy(), np.array(want, np.float32), rtol=1e-5, atol=1e-5)
    assert torch.equal(t0["boxes_world"][:, 2:], torch.tensor([[0.5, 0.7], [0.5, 0.7]]))
    assert t0["keypoints"] is None and t0["calib"]["intrinsic"] is Ks
    # world_pos format: entries with < 2 values are skipped
    assert torch.equal(ds.targets_per_frame[1]["centers_world"], torch.tensor([[1.5, -2.0]]))
    # unparsable JSON -> no targets (the reference logs and continues)
    assert ds.targets_per_frame[2]["boxes_world"].shape == (0, 4)
    # single-point helper agrees with the reference recipe
    assert _pixel_to_world(700.0, 500.0, Ks[2], Rts[2]) == pytest.approx(_ref_pixel_to_world(700.0, 500.0, Ks[2], Rts[2]),
                                                                        rel=1e-6)


def test_dataset_items_and_collate(wildtrack_root):
    ds = WildtrackDataset(_cfg(wildtrack_root))
    torch.manual_seed(3)
    it = ds[1]
    assert it["images"].shape == (7, 3) + IMG_HW and it["images"].dtype == torch.float32
    assert it["meta"]["frame_idx"] == 1 and it["meta"]["paths"][6].endswith("C7/00000005.png")
    torch.manual_seed(3)
    assert torch.equal(ds[1]["images"], it["images"])  # augmentation draws from torch's global generator
    b = collate_fn([ds[0], ds[2]])
    assert b["images"].shape == (2, 7, 3) + IMG_HW
    assert len(b["calib"]["intrinsic"]) == 2 and len(b["calib"]["intrinsic"][0]) == 7
    assert [m["frame_idx"] for m in b["meta"]] == [0, 2]
    u8 = WildtrackDataset(_cfg(wildtrack_root), images_uint8=True)
    x = u8[0]["images"]
    assert x.shape == (7,) + IMG_HW + (3,) and x.dtype == torch.uint8


def test_missing_layout_raises(tmp_path):
    with pytest.raises(FileNotFoundError):
        WildtrackDataset(_cfg(tmp_path))


def test_to_tensor_normalize_known_answer():
    arr = np.arange(0, 256, dtype=np.uint8)[:240].reshape(8, 10, 3)
    img = Image.fromarray(arr)
    got = T.Normalize(T.IMAGENET_MEAN, T.IMAGENET_STD)(T.ToTensor()(img)).numpy()
    x = arr.transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    want = (x - np.array(T.IMAGENET_MEAN, np.float32)[:, None, None]) / np.array(T.IMAGENET_STD, np.float32)[:, None, None]
    assert np.array_equal(got.view(np.uint32), want.astype(np.float32).view(np.uint32))


def test_resize_and_jitter_semantics():
    from PIL import ImageEnhance
    rng = np.random.default_rng(1)
    img = Image.fromarray(rng.integers(0, 256, size=(40, 60, 3), dtype=np.uint8))
    r = T.Resize((20, 33))(img)
    assert r.size == (33, 20) and np.array_equal(np.array(r), np.array(img.resize((33, 20), Image.BILINEAR)))
    cj = T.ColorJitter(brightness=0.2, contrast=0.2, saturation=0.2, hue=0.05)
    assert cj.brightness == (0.8, 1.2) and cj.hue == (-0.05, 0.05)
    torch.manual_seed(7)
    got = np.array(cj(img))
    torch.manual_seed(7)
    order = torch.randperm(4).tolist()
    f = [float(torch.empty(1).uniform_(0.8, 1.2)) for _ in range(3)] + [float(torch.empty(1).uniform_(-0.05, 0.05))]
    want = img
    for k in order:
        if k == 0:
            want = ImageEnhance.Brightness(want).enhance(f[0])
        elif k == 1:
            want = ImageEnhance.Contrast(want).enhance(f[1])
        elif k == 2:
            want = ImageEnhance.Color(want).enhance(f[2])
        else:
            h, s, v = want.convert("HSV").split()
            hh = np.array(h, dtype=np.uint8)
            with np.errstate(over="ignore"):
                hh += np.array(f[3] * 255).astype(np.uint8)
            want = Image.merge("HSV", (Image.fromarray(hh, "L"), s, v)).convert("RGB")
    assert np.array_equal(got, np.array(want))
    ra = T.RandomApply([lambda im: "applied"], p=0.5)
    torch.manual_seed(0)
    draws = [float(torch.rand(1)) for _ in range(20)]
    torch.manual_seed(0)
    assert [ra(img) == "applied" for _ in range(20)] == [d <= 0.5 for d in draws]


@pytest.mark.gpu
def test_normalize_on_device_bit_exact():
    rng = np.random.default_rng(5)
    for shape in [(2, 3, 54, 96), (1, 1, 7, 9), (1, 2, 5, 3)]:  # vector path, odd HW (scalar path)
        arr = rng.integers(0, 256, size=shape + (3,), dtype=np.uint8)
        got = T.normalize_on_device(torch.from_numpy(arr).cuda()).cpu()
        cpu = torch.stack([torch.stack([T.Normalize(T.IMAGENET_MEAN, T.IMAGENET_STD)(
            T.ToTensor()(Image.fromarray(arr[b, v]))) for v in range(shape[1])]) for b in range(shape[0])])
        assert got.shape == cpu.shape
        assert torch.equal(got.view(torch.int32), cpu.view(torch.int32))


@pytest.mark.gpu
def test_wildtrack_batch_through_bevnet(wildtrack_root):
    """The reference's train-loop shape: DataLoader(collate_fn) batch -> BEVNet forward + loss + backward."""
    from models.model_wrapper import BEVNet
    cfg = _cfg(wildtrack_root)
    cfg["MODEL"] = {"BACKBONE": "resnet18", "PRETRAINED": False, "FEAT_DIM": 32, "OUT_INDEX": 2,
                    "BEV_SIZE": [32, 24, 72], "BEV_BOUNDS": [-24.0, 24.0, -7.2, 7.2], "BEV_PROJ_CH": 32}
    ds = WildtrackDataset(cfg, images_uint8=True)
    dl = torch.utils.data.DataLoader(ds, batch_size=2, shuffle=False, collate_fn=collate_fn)
    batch = next(iter(dl))
    images = T.normalize_on_device(batch["images"].cuda())
    assert images.shape == (2, 7, 3) + IMG_HW
    calib = {k: [[m.cuda() for m in per] for per in batch["calib"][k]] for k in ("intrinsic", "extrinsic")}
    net = BEVNet(cfg).cuda().train()
    out = net({"images": images, "calib": calib})
    assert out["heatmap_logits"].shape[-2:] == (24, 72)
    losses = net.loss(out, [{k: (v.cuda() if torch.is_tensor(v) else v) for k, v in t.items() if k != "calib"}
                            for t in batch["targets"]], cfg.get("LOSS", {}))
    total = losses["total_loss"]
    assert math.isfinite(float(total))
    total.backward()
    assert any(p.grad is not None and torch.isfinite(p.grad).all() for p in net.parameters())
