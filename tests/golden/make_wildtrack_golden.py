"""Golden fixtures for the Wildtrack data path, recorded from the reference itself.

Run ONLY in the build container, where the read-only reference tree exists:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_wildtrack_golden.py

The reference's `data/wildtrack_loader.py` imports `torchvision.transforms` at module scope (:8, and
`data/transforms.py:1`), and torchvision is absent from this image.  The helpers pinned here are pure torch +
stdlib and never touch it, so a stub module is registered under `torchvision` / `torchvision.transforms` for the
import alone: every attribute access on the stub raises, so no recorded value can come from it (the transform
pipeline, `build_transforms`, is NOT recorded; `data/transforms.py` is pinned by its own known answers).

Recorded (reference file:line):
  * `_parse_float_list` (:47-61) on separator / junk-token strings;
  * `_load_camera_xml` (:94-136) on XML texts covering every tag family (K / intrinsic / camera_matrix <data>,
    RT, R + T, missing -> default K and identity Rt, nested OpenCV text);
  * `_discover_camera_xmls` (:139-151) on a directory of file names;
  * `_load_wildtrack_calibrations` (:154-247) on synthetic calibration trees: the 7-camera Wildtrack order with
    intrinsic_zero / extrinsic, OpenCV camera_matrix intrinsics and rvec / tvec extrinsics in centimetres (the
    >100 "millimetre" rule), RT and R + T extrinsics, a missing camera, and the non-7 naming rule (views = 3);
  * `_rodrigues` (:404-415) on axis-angle vectors incl. theta < 1e-8;
  * `_compute_homography` / `_compute_img_to_world_homography` / `_pixel_to_world` (:18-44) on a grid of pixels;
  * `WildtrackDataset._prepare_targets` (:311-363) world centres and boxes for three annotation files (the list
    of people with per-view boxes, the {'annotations': [{'world_pos'}]} form, an unparsable file), called on an
    instance built without __init__ (which would build the torchvision transforms) -- only the attributes
    `_prepare_targets` reads are set.

Floats are stored as their float32 bit patterns (uint32) so the test compares bit for bit.  Inputs are this
script's own synthetic files (written into a temporary tree and also stored as text in the fixture), never the
reference's data.  Output: tests/golden/wildtrack_cases.json.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/project"
OUT = os.path.join(HERE, "wildtrack_cases.json")


class _Stub(types.ModuleType):
    def __getattr__(self, name):  # any use of torchvision by a recorded function would fail loudly here
        if name.startswith("__"):  # module protocol probes (inspect, importlib): plain "absent"
            raise AttributeError(name)
        raise RuntimeError(f"torchvision stub: attribute {name!r} used; recording aborted")


def _import_reference():
    import torch  # noqa: F401  (imported before the stub exists: torch's own optional torchvision probes see none)
    tv = _Stub("torchvision")
    tvt = _Stub("torchvision.transforms")
    tv.transforms = tvt
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = tvt
    sys.path.insert(0, REF)
    import data.wildtrack_loader as wl  # noqa: E402  (reference)
    return wl


def bits(t) -> list:
    a = np.ascontiguousarray(np.asarray(t, dtype=np.float32))
    return {"shape": list(a.shape), "u32": a.view(np.uint32).reshape(-1).tolist()}


# ---------------------------------------------------------------- synthetic inputs (this script's own)
def rig(v):
    K = np.array([[1700.0 + 20 * v, 0.0, 960.0 - 5 * v], [0.0, 1690.0 + 10 * v, 540.0 + 3 * v], [0.0, 0.0, 1.0]])
    rvec = np.array([1.7 + 0.05 * v, 0.4 - 0.1 * v, -0.3 + 0.07 * v])
    tvec = np.array([-500.0 + 80 * v, 45.0 - 10 * v, 990.0 + 15 * v])
    return K, rvec, tvec


def opencv_matrix(tag, M):
    rows, cols = M.shape
    data = " ".join(f"{x:.10e}" for x in M.reshape(-1))
    return (f'<{tag} type_id="opencv-matrix">\n  <rows>{rows}</rows>\n  <cols>{cols}</cols>\n  <dt>d</dt>\n'
            f"  <data>\n    {data}</data></{tag}>\n")


def intrinsic_xml(K):
    return ('<?xml version="1.0"?>\n<opencv_storage>\n' + opencv_matrix("camera_matrix", K) +
            opencv_matrix("distortion_coefficients", np.array([[-0.3], [0.1], [0.0], [0.0], [0.0]])) +
            "</opencv_storage>\n")


def rvec_xml(rvec, tvec, row=False):
    if row:
        return (f'<?xml version="1.0"?>\n<opencv_storage>\n<rvec>{" ".join(repr(float(x)) for x in rvec)}</rvec>\n'
                f'<tvec>{" ".join(repr(float(x)) for x in tvec)}</tvec>\n</opencv_storage>\n')
    return ('<?xml version="1.0"?>\n<opencv_storage>\n' + opencv_matrix("rvec", np.asarray(rvec).reshape(3, 1)) +
            opencv_matrix("tvec", np.asarray(tvec).reshape(3, 1)) + "</opencv_storage>\n")


CAMERA_XMLS = {
    "k_rt": "<c><K>2 0 3 0 4 5 0 0 1</K><RT>1 0 0 10 0 1 0 20 0 0 1 30</RT></c>",
    "rot_trans": "<c><rotation>0 -1 0 1 0 0 0 0 1</rotation><translation>1;2;3</translation></c>",
    "empty": "<c/>",
    "nested": "<c><A><x>1</x><x>2</x><x>3</x><x>4 5 6</x><x>7 8 9</x></A><R>1,0,0;0,1,0;0,0,1</R><T>0.5 junk 1.5 2.5</T></c>",
    "opencv": '<?xml version="1.0"?>\n<opencv_storage>\n' + opencv_matrix("intrinsic", np.array(
        [[1234.5, 0.0, 955.25], [0.0, 1233.75, 541.0], [0.0, 0.0, 1.0]])) + opencv_matrix("ExtrinsicMatrix", np.array(
        [[0.6, -0.8, 0.0, 1.25], [0.8, 0.6, 0.0, -2.5], [0.0, 0.0, 1.0, 7.75]])) + "</opencv_storage>\n",
    "short_rt": "<c><MatrixK>1 0 0 0 1 0 0 0 1</MatrixK><RT>1 2 3</RT><R>1 0 0 0 1 0 0 0 1</R><t>4 5 6</t></c>",
}

FLOAT_LISTS = ["1, 2;3\n4\t5  six 7e-1", "", "  ;;,, ", "-1.5e3 nan 0x10 +2 .5", "1e400 -0 3"]

DISCOVER_NAMES = ["cam-C2.xml", "x-3.xml", "cam_C4.xml", "C1_extra.xml", "4.xml", "calibC5.xml", "sub/C6.xml"]


def people():
    return [
        {"personID": 0, "positionID": 11, "views": [
            {"viewNum": 0, "xmin": 100, "ymin": 300, "xmax": 160, "ymax": 620},
            {"viewNum": 3, "xmin": 880, "ymin": 200, "xmax": 950, "ymax": 530},
            {"viewNum": 6, "xmin": 1200, "ymin": 400, "xmax": 1290, "ymax": 800}]},
        {"personID": 1, "positionID": 12, "views": [
            {"viewNum": 2, "xmin": 500, "ymin": 100, "xmax": 540, "ymax": 333},
            {"viewNum": 9, "xmin": 1, "ymin": 1, "xmax": 2, "ymax": 2},
            {"viewNum": 4, "xmin": None, "ymin": 1, "xmax": 2, "ymax": 2}]},
        {"personID": 2, "positionID": 13, "views": [{"viewNum": 1, "xmin": 10, "ymin": 10}]},
        {"personID": 3, "positionID": 14, "views": [
            {"viewNum": 5, "xmin": 300.5, "ymin": 50, "xmax": 341.25, "ymax": 910.75},
            {"viewNum": 1, "xmin": 1500, "ymin": 20, "xmax": 1560, "ymax": 700}]},
        {"personID": 4, "positionID": 15, "views": []},
    ]


ANNOTATIONS = {
    "00000000": json.dumps(people()),
    "00000005": json.dumps({"annotations": [{"world_pos": [1.5, -2.0]}, {"world_pos": [3.0]},
                                            {"world_pos": [0.1, 0.2, 0.0]}]}),
    "00000010": "{ not json",
    "00000015": json.dumps([]),
}


def calibration_trees():
    """name -> (views, {relative path: text}); every tree is written under <tmp>/<name>/."""
    trees = {}
    files = {}
    for v, name in enumerate(["CVLab1", "CVLab2", "CVLab3", "CVLab4", "IDIAP1", "IDIAP2", "IDIAP3"]):
        K, rvec, tvec = rig(v)
        files[f"intrinsic_zero/intr_{name}.xml"] = intrinsic_xml(K)
        files[f"extrinsic/extr_{name}.xml"] = rvec_xml(rvec, tvec, row=(v % 2 == 1))
    trees["wildtrack7"] = (7, files)
    # intrinsic_original preferred over intrinsic_zero; RT / R+T extrinsics; metres kept (|t| <= 100);
    # camera IDIAP3 missing entirely (default K, identity Rt)
    files = {}
    for v, name in enumerate(["CVLab1", "CVLab2", "CVLab3", "CVLab4", "IDIAP1", "IDIAP2"]):
        K, rvec, tvec = rig(v)
        files[f"intrinsic_original/{name}.xml"] = intrinsic_xml(K * 0.5 + np.eye(3) * 0.5)
        files[f"intrinsic_zero/{name}.xml"] = intrinsic_xml(np.eye(3))
        if v % 3 == 0:
            files[f"extrinsic/{name}.xml"] = ("<c><RT>" + " ".join(f"{x:.9g}" for x in np.hstack(
                [np.eye(3)[[1, 2, 0]], np.array([[1.5 + v], [-2.0], [30.0]])]).reshape(-1)) + "</RT></c>")
        elif v % 3 == 1:
            files[f"extrinsic/{name}.xml"] = (f"<c><R>0 0 1 1 0 0 0 1 0</R><T>{v}.25 -3.5 {250.0 + v}</T></c>")
        else:
            files[f"extrinsic/{name}.xml"] = "<c><nothing/></c>"
    trees["variants7"] = (7, files)
    # non-7 views: names from the files (CVLab* sorted, then IDIAP*), padded with Cam{i}
    files = {"extrinsic/extr_IDIAP2.xml": rvec_xml(np.zeros(3), np.array([1.0, 2.0, 3.0])),
             "intr_CVLab3.xml": intrinsic_xml(np.diag([5.0, 6.0, 1.0])),
             "intr_cvlab1.xml": intrinsic_xml(np.diag([7.0, 8.0, 1.0]))}
    trees["views4"] = (4, files)
    return trees


def main():
    wl = _import_reference()
    import torch

    out = {"torch": torch.__version__, "reference": "project/data/wildtrack_loader.py",
           "inputs": {"camera_xmls": CAMERA_XMLS, "float_lists": FLOAT_LISTS, "discover_names": DISCOVER_NAMES,
                      "annotations": ANNOTATIONS}}
    out["float_lists"] = [wl._parse_float_list(s) for s in FLOAT_LISTS]
    out["float_lists"] = [[repr(x) for x in vals] for vals in out["float_lists"]]

    with tempfile.TemporaryDirectory() as tmp:
        tmp = Path(tmp)
        cams = {}
        for name, text in CAMERA_XMLS.items():
            p = tmp / f"{name}.xml"
            p.write_text(text)
            K, Rt = wl._load_camera_xml(p)
            cams[name] = {"K": bits(K), "Rt": bits(Rt)}
        out["camera_xml"] = cams

        d = tmp / "discover"
        for n in DISCOVER_NAMES:
            (d / n).parent.mkdir(parents=True, exist_ok=True)
            (d / n).write_text("<c/>")
        found = wl._discover_camera_xmls(d, 7)
        out["discover"] = [None if f is None else str(f.relative_to(d)) for f in found]

        calib = {}
        trees = calibration_trees()
        out["inputs"]["calibration_trees"] = {k: {"views": v, "files": f} for k, (v, f) in trees.items()}
        for tname, (views, files) in trees.items():
            root = tmp / tname
            for rel, text in files.items():
                (root / rel).parent.mkdir(parents=True, exist_ok=True)
                (root / rel).write_text(text)
            Ks, Rts = wl._load_wildtrack_calibrations(root, views)
            calib[tname] = {"K": [bits(k) for k in Ks], "Rt": [bits(r) for r in Rts]}
        out["calibrations"] = calib

        rvecs = [[1.7, 0.4, -0.3], [0.0, 0.0, 0.0], [1e-9, 0.0, 0.0], [3.1, -0.2, 0.05], [-0.5, 2.0, 1.25],
                 [0.0, 0.0, 3.14159265]]
        out["inputs"]["rvecs"] = rvecs
        out["rodrigues"] = [bits(wl._rodrigues(torch.tensor(r, dtype=torch.float32).view(3, 1))) for r in rvecs]

        # pixel -> world for every camera of the 7-camera tree, on a grid (ground points, horizon, w ~ 0)
        Ks7 = [torch.from_numpy(np.frombuffer(np.array(c["u32"], np.uint32).tobytes(), np.float32).reshape(3, 3))
               for c in calib["wildtrack7"]["K"]]
        Rts7 = [torch.from_numpy(np.frombuffer(np.array(c["u32"], np.uint32).tobytes(), np.float32).reshape(4, 4))
                for c in calib["wildtrack7"]["Rt"]]
        us = [0.0, 1.5, 333.25, 959.5, 1919.0, 2500.0]
        vs = [0.0, 100.0, 540.0, 777.75, 1079.0]
        out["inputs"]["pixels"] = {"u": us, "v": vs}
        p2w = []
        for K, Rt in zip(Ks7, Rts7):
            H = wl._compute_homography(K, Rt)
            Hi = wl._compute_img_to_world_homography(K, Rt)
            pts = []
            for u in us:
                for v in vs:
                    r = wl._pixel_to_world(u, v, K, Rt)
                    pts.append(None if r is None else [repr(r[0]), repr(r[1])])
            p2w.append({"H": bits(H), "H_i2w": bits(Hi), "world": pts})
        out["pixel_to_world"] = p2w
        # a camera whose ground homography is singular (optical axis in the ground plane's direction)
        Ks = torch.eye(3)
        Rts = torch.eye(4)
        Rts[:3, :3] = torch.tensor([[1.0, 0, 0], [0, 0, 1], [0, 1, 0]])  # r2 = (0,0,1): [r1 r2 t] rank-deficient
        Rts[:3, 3] = torch.tensor([0.0, 0.0, 0.0])
        out["singular"] = {"K": bits(Ks), "Rt": bits(Rts), "H_i2w": bits(wl._compute_img_to_world_homography(Ks, Rts)),
                           "world": [None if (r := wl._pixel_to_world(u, v, Ks, Rts)) is None else [repr(r[0]), repr(r[1])]
                                     for u, v in ((0.0, 0.0), (10.0, 5.0), (0.5, 0.25))]}

        # _prepare_targets on the 7-camera calibration, without __init__ (no transforms)
        ann = tmp / "annotations_positions"
        ann.mkdir()
        for stem, text in ANNOTATIONS.items():
            (ann / f"{stem}.json").write_text(text)
        ds = wl.WildtrackDataset.__new__(wl.WildtrackDataset)
        ds.frame_files = [f"{s}.png" for s in sorted(ANNOTATIONS)] + ["00000020.png"]  # last: no annotation file
        ds.intrinsics = [Ks7 for _ in ds.frame_files]
        ds.extrinsics = [Rts7 for _ in ds.frame_files]
        ds.annotations_dir = ann
        ds.default_box_wh = (0.6, 0.45)
        ds.targets_per_frame = []
        ds._prepare_targets()
        out["inputs"]["frame_files"] = ds.frame_files
        out["inputs"]["default_box_wh"] = list(ds.default_box_wh)
        out["targets"] = [{"centers_world": bits(t["centers_world"]), "boxes_world": bits(t["boxes_world"])}
                          for t in ds.targets_per_frame]

    with open(OUT, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(f"wrote {OUT}: {len(out['targets'])} frames, {len(out['calibrations'])} calibration trees")


if __name__ == "__main__":
    main()
