"""Wildtrack dataset -- drop-in for project/data/wildtrack_loader.py.

Same surface as the reference: `WildtrackDataset(cfg)` (wildtrack_loader.py:250-386) returning
`{'images': [V, 3, H, W] f32, 'calib': {'intrinsic': [K]*V, 'extrinsic': [Rt]*V}, 'targets':
{'boxes_world', 'centers_world', 'keypoints', 'calib'}, 'meta': {'frame_idx', 'paths'}}` per frame,
`collate_fn` (:389-401), and the calibration / annotation helpers the reference defines at module
level (`_parse_float_list` :47, `_try_get_matrix` :70, `_load_camera_xml` :94,
`_discover_camera_xmls` :139, `_load_wildtrack_calibrations` :154, `_pixel_to_world` :35,
`_rodrigues` :404), with the reference's rules:

* OpenCV-XML matrices under several tag spellings, `<data>` child, raw text or nested text;
* per camera (default Wildtrack order CVLab1-4, IDIAP1-3 when V = 7) an intrinsic XML from
  `intrinsic_original/` (else `intrinsic_zero/`, else the calibration root) and an extrinsic XML
  from `extrinsic/`: RT 3x4, else R + T, else Rodrigues rvec + tvec; missing -> K = diag(1000,
  1000, 1), Rt = I; translation norms above 100 are taken as millimetres and divided by 1000;
* annotation JSON per frame (`annotations_positions/` preferred): either {'annotations':
  [{'world_pos': [x, y]}]} or the Wildtrack list of people whose per-view boxes give a
  ground point (bottom centre) projected through inv(K [r1 r2 t]) and averaged over views;
  boxes_world = centres + LOSS.DEFAULT_BOX_WH.

Differences (documented, not semantic): no torchvision dependency (data/transforms.py restates the
transform pipeline); the inverse homography of each camera is computed once per dataset instead of
once per annotated box (same matrices), and the bottom-centre points of one camera are projected
as one batch (float32 matmul, equal to the per-point product within fp32 rounding);
`images_uint8=True` makes __getitem__ return [V, H, W, 3] uint8 for on-device normalisation
(`data.transforms.normalize_on_device`).

Not on the hot path: this is host I/O that feeds it (JPEG/PNG decode in DataLoader workers).
"""
from __future__ import annotations

import json
import math
import re
import xml.etree.ElementTree as ET
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple

import torch
from PIL import Image

from .transforms import build_transforms

K_TAGS = ["K", "intrinsic", "intrinsics", "camera_matrix", "IntrinsicMatrix", "MatrixK", "A"]
K_TAGS_CALIB = ["K", "intrinsic", "camera_matrix", "IntrinsicMatrix", "MatrixK", "A"]
R_TAGS = ["R", "rotation", "RotationMatrix", "rotation_matrix"]
T_TAGS = ["T", "translation", "TranslationVector", "t"]
RT_TAGS = ["RT", "ExtrinsicMatrix", "Pose", "MatrixRT"]
RVEC_TAGS = ["rvec", "Rodrigues", "rotation_vector"]
TVEC_TAGS = ["tvec", "t", "translation_vector"]
WILDTRACK_CAMERAS = ["CVLab1", "CVLab2", "CVLab3", "CVLab4", "IDIAP1", "IDIAP2", "IDIAP3"]

_SEP = re.compile(r"[\,;\n\t]+")


def _default_K() -> torch.Tensor:
    K = torch.eye(3, dtype=torch.float32)
    K[0, 0] = K[1, 1] = 1000.0
    return K


# ---------------------------------------------------------------------------
# geometry helpers (wildtrack_loader.py:18-44)
# ---------------------------------------------------------------------------
def _compute_homography(K: torch.Tensor, Rt: torch.Tensor) -> torch.Tensor:
    """K @ [r1 r2 t] (world plane z = 0 -> pixels), float32."""
    G = torch.eye(3, dtype=torch.float32)
    G[:, :2] = Rt[:3, :2]
    G[:, 2:3] = Rt[:3, 3:4]
    return K @ G


def _compute_img_to_world_homography(K: torch.Tensor, Rt: torch.Tensor) -> torch.Tensor:
    H = _compute_homography(K, Rt)
    try:
        return torch.linalg.inv(H)
    except Exception:  # singular: the reference's pinv fallback
        return torch.linalg.pinv(H)


def _project_to_world(H_i2w: torch.Tensor, uv: torch.Tensor) -> List[Optional[Tuple[float, float]]]:
    """[N, 2] pixels -> per point (x, y) metres on z = 0, or None where w is NaN or |w| < 1e-8."""
    if uv.numel() == 0:
        return []
    uv1 = torch.cat([uv.to(torch.float32), torch.ones(uv.shape[0], 1, dtype=torch.float32)], dim=1)
    xyw = H_i2w @ uv1.T  # [3, N]
    out: List[Optional[Tuple[float, float]]] = []
    for x, y, w in zip(xyw[0].tolist(), xyw[1].tolist(), xyw[2].tolist()):
        if not (w == w) or abs(w) < 1e-8:
            out.append(None)
            continue
        # float32 divisions, like the reference's float(xyw[0, 0] / w) on tensors
        wt = torch.tensor(w, dtype=torch.float32)
        out.append((float(torch.tensor(x, dtype=torch.float32) / wt), float(torch.tensor(y, dtype=torch.float32) / wt)))
    return out


def _pixel_to_world(u: float, v: float, K: torch.Tensor, Rt: torch.Tensor) -> Optional[Tuple[float, float]]:
    return _project_to_world(_compute_img_to_world_homography(K, Rt), torch.tensor([[u, v]]))[0]


# ---------------------------------------------------------------------------
# XML parsing (wildtrack_loader.py:47-151)
# ---------------------------------------------------------------------------
def _parse_float_list(text: Optional[str]) -> List[float]:
    """Floats of a comma / semicolon / whitespace separated string; other tokens are skipped."""
    if text is None:
        return []
    vals = []
    for tok in _SEP.sub(" ", text).strip().split(" "):
        if not tok:
            continue
        try:
            vals.append(float(tok))
        except ValueError:
            continue
    return vals


def _reshape(vals: List[float], rows: int, cols: int) -> torch.Tensor:
    """The first rows*cols values as a float32 [rows, cols] matrix (extra values are ignored)."""
    n = rows * cols
    if n > len(vals):
        raise ValueError(f"Not enough values to reshape: need {n}, got {len(vals)}")
    return torch.tensor(vals[:n], dtype=torch.float32).view(rows, cols)


def _try_get_matrix(root: ET.Element, tag_names: List[str], shape: Tuple[int, int]) -> Optional[torch.Tensor]:
    """First matrix found under any tag name: its <data> child, its own text, or all nested text."""
    rows, cols = shape
    need = rows * cols
    for name in tag_names:
        for elem in root.findall(f".//{name}"):
            data = elem.find("data")
            sources = []
            if data is not None and data.text is not None:
                sources.append(data.text)
            if elem.text is not None:
                sources.append(elem.text)
            sources.append(" ".join(e.text or "" for e in elem.iter()))
            for src in sources:
                vals = _parse_float_list(src)
                if len(vals) >= need:
                    return _reshape(vals, rows, cols)
    return None


def _rt44(Rt34: Optional[torch.Tensor]) -> torch.Tensor:
    Rt = torch.eye(4, dtype=torch.float32)
    if Rt34 is not None:
        Rt[:3, :4] = Rt34
    return Rt


def _load_camera_xml(xml_path: Path) -> Tuple[torch.Tensor, torch.Tensor]:
    """K (3x3) and Rt (4x4) from one camera XML (RT, or R + T; defaults as the reference)."""
    root = ET.parse(str(xml_path)).getroot()
    K = _try_get_matrix(root, K_TAGS, (3, 3))
    Rt34 = _try_get_matrix(root, RT_TAGS, (3, 4))
    if Rt34 is None:
        R = _try_get_matrix(root, R_TAGS, (3, 3))
        t = _try_get_matrix(root, T_TAGS, (3, 1))
        Rt34 = torch.cat([R, t], dim=1) if (R is not None and t is not None) else None
    return (K if K is not None else _default_K()), _rt44(Rt34)


def _discover_camera_xmls(calib_dir: Path, views: int) -> List[Optional[Path]]:
    """XML per camera 1..views: a stem containing the token C{i} (any case), else the token {i}."""
    if not calib_dir.exists():
        return [None] * views
    xmls = list(calib_dir.rglob("*.xml"))
    out: List[Optional[Path]] = []
    for i in range(1, views + 1):
        hits = [p for p in xmls if re.search(fr"(^|[^\w])C{i}([^\w]|$)", p.stem, flags=re.IGNORECASE)]
        if not hits:
            hits = [p for p in xmls if re.search(fr"(^|[^\w]){i}([^\w]|$)", p.stem)]
        out.append(hits[0] if hits else None)
    return out


def _rodrigues(rvec: torch.Tensor) -> torch.Tensor:
    """Rotation matrix of an axis-angle vector: I + sin(th) [k]x + (1 - cos(th)) [k]x^2 (float32)."""
    rv = rvec.reshape(-1).to(torch.float32)
    theta = torch.norm(rv).item()
    if theta < 1e-8:
        return torch.eye(3, dtype=torch.float32)
    k = rv / theta
    kx, ky, kz = (float(v) for v in k.tolist())
    S = torch.tensor([[0.0, -kz, ky], [kz, 0.0, -kx], [-ky, kx, 0.0]], dtype=torch.float32)
    return torch.eye(3, dtype=torch.float32) + math.sin(theta) * S + (1.0 - math.cos(theta)) * (S @ S)


def _extrinsic_from_root(root: ET.Element) -> Optional[torch.Tensor]:
    """3x4 [R | t]: RT, else R + T, else Rodrigues rvec + tvec (3x1 or 1x3)."""
    Rt34 = _try_get_matrix(root, RT_TAGS, (3, 4))
    if Rt34 is not None:
        return Rt34
    R = _try_get_matrix(root, R_TAGS, (3, 3))
    t = _try_get_matrix(root, T_TAGS, (3, 1))
    if R is not None and t is not None:
        return torch.cat([R, t], dim=1)
    rvec = _try_get_matrix(root, RVEC_TAGS, (3, 1))
    if rvec is None:
        rvec = _try_get_matrix(root, RVEC_TAGS, (1, 3))
    tvec = _try_get_matrix(root, TVEC_TAGS, (3, 1))
    if tvec is None:
        tvec = _try_get_matrix(root, TVEC_TAGS, (1, 3))
    if rvec is None or tvec is None:
        return None
    return torch.cat([_rodrigues(rvec), tvec.reshape(3, 1)], dim=1)


def _camera_names(intr_dir: Path, extr_dir: Path, views: int) -> List[str]:
    if views == 7:
        return list(WILDTRACK_CAMERAS)
    names = set()
    for p in list(intr_dir.rglob("*.xml")) + list(extr_dir.rglob("*.xml")):
        m = re.search(r"(CVLab\d+|IDIAP\d+)", p.stem, flags=re.IGNORECASE)
        if m:
            names.add(m.group(1))
    cams = sorted(n for n in names if n.lower().startswith("cvlab")) + \
        sorted(n for n in names if n.lower().startswith("idiap"))
    if len(cams) < views:
        cams += [f"Cam{i}" for i in range(len(cams) + 1, views + 1)]
    return cams[:views]


def _load_wildtrack_calibrations(calib_root: Path, views: int) -> Tuple[List[torch.Tensor], List[torch.Tensor]]:
    """Per-camera K [3, 3] and Rt [4, 4] from the Wildtrack calibration tree (wildtrack_loader.py:154-247)."""
    calib_root = Path(calib_root)
    if (calib_root / "intrinsic_original").exists():
        intr_dir = calib_root / "intrinsic_original"
    elif (calib_root / "intrinsic_zero").exists():
        intr_dir = calib_root / "intrinsic_zero"
    else:
        intr_dir = calib_root
    extr_dir = calib_root / "extrinsic" if (calib_root / "extrinsic").exists() else calib_root
    intr_xmls = list(intr_dir.rglob("*.xml"))
    extr_xmls = list(extr_dir.rglob("*.xml"))

    Ks: List[torch.Tensor] = []
    Rts: List[torch.Tensor] = []
    for name in _camera_names(intr_dir, extr_dir, views):
        pat = re.compile(name, flags=re.IGNORECASE)
        intr = next((p for p in intr_xmls if pat.search(p.stem)), None)
        extr = next((p for p in extr_xmls if pat.search(p.stem)), None)
        K = None
        if intr is None:
            print(f"[WildtrackDataset] warning: no intrinsic XML for camera {name}; default K")
        else:
            K = _try_get_matrix(ET.parse(str(intr)).getroot(), K_TAGS_CALIB, (3, 3))
            if K is None:
                print(f"[WildtrackDataset] warning: no K parsed from {intr}; default K")
        Ks.append(K if K is not None else _default_K())

        Rt34 = None
        if extr is None:
            print(f"[WildtrackDataset] warning: no extrinsic XML for camera {name}; identity Rt")
        else:
            Rt34 = _extrinsic_from_root(ET.parse(str(extr)).getroot())
            if Rt34 is None:
                print(f"[WildtrackDataset] warning: no Rt parsed from {extr}; identity Rt")
        Rt = _rt44(Rt34)
        if Rt34 is not None and float(torch.norm(Rt[:3, 3])) > 100.0:
            Rt[:3, 3] = Rt[:3, 3] / 1000.0  # translation taken as millimetres -> metres
        Rts.append(Rt)
    return Ks, Rts


# ---------------------------------------------------------------------------
# annotations (wildtrack_loader.py:311-363)
# ---------------------------------------------------------------------------
def _frame_centres(data: Any, H_i2w: List[torch.Tensor]) -> List[List[float]]:
    """World centres of one frame's annotation JSON (either reference format)."""
    centres: List[List[float]] = []
    if isinstance(data, dict) and "annotations" in data:
        for ann in data["annotations"]:
            wp = ann.get("world_pos", None)
            if wp and len(wp) >= 2:
                centres.append([float(wp[0]), float(wp[1])])
        return centres
    if not isinstance(data, list):
        return centres
    # gather every valid per-view bottom-centre point, project per camera in one batch
    owner: List[Tuple[int, int]] = []  # (person, camera)
    pts: Dict[int, List[Tuple[float, float]]] = {}
    for pi, person in enumerate(data):
        for view in person.get("views", []):
            vnum = int(view.get("viewNum", -1))
            if vnum < 0 or vnum >= len(H_i2w):
                continue
            box = [view.get(k, None) for k in ("xmin", "xmax", "ymin", "ymax")]
            if None in box:
                continue
            u = 0.5 * (float(box[0]) + float(box[1]))
            pts.setdefault(vnum, []).append((u, float(box[3])))
            owner.append((pi, vnum))
    world: Dict[int, List[Optional[Tuple[float, float]]]] = {
        v: _project_to_world(H_i2w[v], torch.tensor(p, dtype=torch.float64)) for v, p in pts.items()}
    cursor = {v: 0 for v in world}
    per_person: Dict[int, List[Tuple[float, float]]] = {}
    for pi, v in owner:
        wp = world[v][cursor[v]]
        cursor[v] += 1
        if wp is not None:
            per_person.setdefault(pi, []).append(wp)
    for pi in sorted(per_person):
        ps = per_person[pi]
        centres.append([sum(p[0] for p in ps) / len(ps), sum(p[1] for p in ps) / len(ps)])
    return centres


class WildtrackDataset(torch.utils.data.Dataset):
    """Multi-view Wildtrack frames (wildtrack_loader.py:250-386)."""

    def __init__(self, cfg: Dict[str, Any], images_uint8: bool = False):
        self.cfg = cfg
        self.data_root = Path(cfg["DATA"]["DATA_ROOT"]).resolve()
        self.views = int(cfg["DATA"]["VIEWS"])
        _, H, W = cfg["DATA"]["IMG_SIZE"]
        self.img_size = (int(H), int(W))
        self.images_uint8 = bool(images_uint8)
        self.transform = build_transforms(img_size=self.img_size, normalize=not self.images_uint8)
        wh = cfg.get("LOSS", {}).get("DEFAULT_BOX_WH", [0.6, 0.6])
        self.default_box_wh = (float(wh[0]), float(wh[1]))

        img_root = self.data_root / "Image_subsets"
        if not img_root.exists():
            raise FileNotFoundError(f"image root not found: {img_root}")
        self.cam_dirs: List[Path] = []
        for i in range(1, self.views + 1):
            d = img_root / f"C{i}"
            if not d.exists():
                raise FileNotFoundError(f"camera folder not found: {d}")
            self.cam_dirs.append(d)
        self.frame_files = sorted(p.name for p in self.cam_dirs[0].iterdir() if p.is_file())
        if not self.frame_files:
            raise FileNotFoundError("no image files found")

        calib_dir = next((d for d in (self.data_root / "Calibration", self.data_root / "Calibrations",
                                      self.data_root / "calibration") if d.exists()), None)
        if calib_dir is None:
            raise FileNotFoundError("calibration directory not found (tried Calibration/Calibrations/calibration)")
        Ks, Rts = _load_wildtrack_calibrations(calib_dir, self.views)
        # static per camera: every frame shares the same lists (as the reference)
        self.intrinsics = [Ks for _ in self.frame_files]
        self.extrinsics = [Rts for _ in self.frame_files]

        self.annotations_dir = next((d for d in (self.data_root / "annotations_positions",
                                                 self.data_root / "Annotations",
                                                 self.data_root / "annotations") if d.exists()), None)
        self.targets_per_frame: List[Dict[str, Any]] = []
        self._prepare_targets()

    def __len__(self) -> int:
        return len(self.frame_files)

    def _prepare_targets(self) -> None:
        Ks0 = self.intrinsics[0] if self.intrinsics else []
        Rts0 = self.extrinsics[0] if self.extrinsics else []
        H_i2w = [_compute_img_to_world_homography(K, Rt) for K, Rt in zip(Ks0, Rts0)]
        w, h = self.default_box_wh
        for idx, fname in enumerate(self.frame_files):
            centres: List[List[float]] = []
            if self.annotations_dir is not None:
                path = self.annotations_dir / (Path(fname).stem + ".json")
                if path.exists():
                    try:
                        with open(path, "r") as f:
                            centres = _frame_centres(json.load(f), H_i2w)
                    except Exception as e:  # the reference logs and keeps the frame unannotated
                        print(f"[WildtrackDataset] failed to parse annotations: {path} ({e})")
                        centres = []
            c = torch.tensor(centres, dtype=torch.float32) if centres else torch.zeros(0, 2)
            if c.numel() > 0:
                boxes = torch.cat([c, torch.tensor([w, h], dtype=torch.float32).repeat(c.shape[0], 1)], dim=1)
            else:
                boxes = torch.zeros(0, 4, dtype=torch.float32)
            self.targets_per_frame.append({
                "boxes_world": boxes,
                "centers_world": c,
                "keypoints": None,
                "calib": {"intrinsic": self.intrinsics[idx], "extrinsic": self.extrinsics[idx]},
            })

    def __getitem__(self, idx: int) -> Dict[str, Any]:
        imgs, paths = [], []
        for v in range(self.views):
            p = self.cam_dirs[v] / self.frame_files[idx]
            imgs.append(self.transform(Image.open(p).convert("RGB")))
            paths.append(str(p))
        calib = {"intrinsic": self.intrinsics[idx], "extrinsic": self.extrinsics[idx]}
        targets = self.targets_per_frame[idx] if idx < len(self.targets_per_frame) else {
            "boxes_world": torch.zeros(0, 4), "centers_world": torch.zeros(0, 2), "keypoints": None, "calib": calib}
        return {"images": torch.stack(imgs, dim=0), "calib": calib, "targets": targets,
                "meta": {"frame_idx": int(idx), "paths": paths}}


def collate_fn(batch: List[Dict[str, Any]]) -> Dict[str, Any]:
    """Stack images to [B, V, ...]; calibrations as List[List[Tensor]] (wildtrack_loader.py:389-401)."""
    batch = [b for b in batch if b is not None]
    return {
        "images": torch.stack([b["images"] for b in batch], dim=0),
        "calib": {"intrinsic": [b["calib"]["intrinsic"] for b in batch],
                  "extrinsic": [b["calib"]["extrinsic"] for b in batch]},
        "targets": [b["targets"] for b in batch],
        "meta": [b["meta"] for b in batch],
    }
