"""Wildtrack data path pinned to the reference itself.

tests/golden/wildtrack_cases.json was recorded by tests/golden/make_wildtrack_golden.py, which imports the
reference's `data/wildtrack_loader.py` (with a raising stub standing in for the torchvision import it never uses
in the recorded helpers) and runs its calibration / annotation helpers on synthetic XML and JSON files that the
script writes and also stores in the fixture.  Here the same files are rebuilt in a temporary tree and this
package's `data/wildtrack_loader.py` must reproduce every recorded value bit for bit (float32 bit patterns):
`_parse_float_list` (:47-61), `_load_camera_xml` (:94-136), `_discover_camera_xmls` (:139-151),
`_load_wildtrack_calibrations` (:154-247), `_rodrigues` (:404-415), `_compute_homography` /
`_compute_img_to_world_homography` / `_pixel_to_world` (:18-44) and `WildtrackDataset._prepare_targets`
(:311-363).
"""
import json
import os
from pathlib import Path

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from data import wildtrack_loader as wl

CASES = json.load(open(os.path.join(GOLDEN, "wildtrack_cases.json")))
INP = CASES["inputs"]


def f32(rec):
    return torch.from_numpy(np.array(rec["u32"], dtype=np.uint32).view(np.float32).reshape(rec["shape"]).copy())


def same_bits(t, rec):
    a = np.ascontiguousarray(t.detach().cpu().numpy().astype(np.float32))
    return list(a.shape) == rec["shape"] and a.view(np.uint32).reshape(-1).tolist() == rec["u32"]


def test_parse_float_list_matches_reference():
    for text, want in zip(INP["float_lists"], CASES["float_lists"]):
        assert [repr(x) for x in wl._parse_float_list(text)] == want, text


@pytest.mark.parametrize("name", sorted(INP["camera_xmls"]))
def test_load_camera_xml_matches_reference(tmp_path, name):
    p = tmp_path / f"{name}.xml"
    p.write_text(INP["camera_xmls"][name])
    K, Rt = wl._load_camera_xml(p)
    assert same_bits(K, CASES["camera_xml"][name]["K"])
    assert same_bits(Rt, CASES["camera_xml"][name]["Rt"])


def test_discover_camera_xmls_matches_reference(tmp_path):
    for n in INP["discover_names"]:
        (tmp_path / n).parent.mkdir(parents=True, exist_ok=True)
        (tmp_path / n).write_text("<c/>")
    got = [None if f is None else str(f.relative_to(tmp_path)) for f in wl._discover_camera_xmls(tmp_path, 7)]
    assert got == CASES["discover"]


@pytest.mark.parametrize("tree", sorted(INP["calibration_trees"]))
def test_calibrations_match_reference(tmp_path, tree):
    spec = INP["calibration_trees"][tree]
    for rel, text in spec["files"].items():
        (tmp_path / rel).parent.mkdir(parents=True, exist_ok=True)
        (tmp_path / rel).write_text(text)
    Ks, Rts = wl._load_wildtrack_calibrations(tmp_path, spec["views"])
    want = CASES["calibrations"][tree]
    assert len(Ks) == len(want["K"]) == spec["views"]
    for v in range(spec["views"]):
        assert same_bits(Ks[v], want["K"][v]), (tree, v)
        assert same_bits(Rts[v], want["Rt"][v]), (tree, v)


def test_rodrigues_matches_reference():
    for r, want in zip(INP["rvecs"], CASES["rodrigues"]):
        assert same_bits(wl._rodrigues(torch.tensor(r, dtype=torch.float32).view(3, 1)), want), r


def test_pixel_to_world_matches_reference():
    Ks = [f32(k) for k in CASES["calibrations"]["wildtrack7"]["K"]]
    Rts = [f32(r) for r in CASES["calibrations"]["wildtrack7"]["Rt"]]
    for K, Rt, want in zip(Ks, Rts, CASES["pixel_to_world"]):
        assert same_bits(wl._compute_homography(K, Rt), want["H"])
        assert same_bits(wl._compute_img_to_world_homography(K, Rt), want["H_i2w"])
        pts = [(u, v) for u in INP["pixels"]["u"] for v in INP["pixels"]["v"]]
        for (u, v), w in zip(pts, want["world"]):
            got = wl._pixel_to_world(u, v, K, Rt)
            assert (got is None) == (w is None), (u, v)
            if got is not None:
                assert [repr(got[0]), repr(got[1])] == w, (u, v)
    s = CASES["singular"]
    K, Rt = f32(s["K"]), f32(s["Rt"])
    assert same_bits(wl._compute_img_to_world_homography(K, Rt), s["H_i2w"])
    for (u, v), w in zip(((0.0, 0.0), (10.0, 5.0), (0.5, 0.25)), s["world"]):
        got = wl._pixel_to_world(u, v, K, Rt)
        assert (got is None) == (w is None) and (got is None or [repr(got[0]), repr(got[1])] == w)


def test_prepare_targets_matches_reference(tmp_path):
    ann = tmp_path / "annotations_positions"
    ann.mkdir()
    for stem, text in INP["annotations"].items():
        (ann / f"{stem}.json").write_text(text)
    Ks = [f32(k) for k in CASES["calibrations"]["wildtrack7"]["K"]]
    Rts = [f32(r) for r in CASES["calibrations"]["wildtrack7"]["Rt"]]
    ds = wl.WildtrackDataset.__new__(wl.WildtrackDataset)
    ds.frame_files = list(INP["frame_files"])
    ds.intrinsics = [Ks for _ in ds.frame_files]
    ds.extrinsics = [Rts for _ in ds.frame_files]
    ds.annotations_dir = ann
    ds.default_box_wh = tuple(INP["default_box_wh"])
    ds.targets_per_frame = []
    ds._prepare_targets()
    assert len(ds.targets_per_frame) == len(CASES["targets"])
    for i, (t, want) in enumerate(zip(ds.targets_per_frame, CASES["targets"])):
        assert same_bits(t["centers_world"], want["centers_world"]), i
        assert same_bits(t["boxes_world"], want["boxes_world"]), i
        assert t["keypoints"] is None and t["calib"]["intrinsic"] is Ks
