"""NeRF dataset ingest: transforms.json + images -> NerfDataset.

Host-side restatement of the reference loader `load_nerf` (src/nerf_loader.cu:260-726) for the
formats the training path consumes: the original NeRF/instant-ngp `transforms.json` (one or more
files), 8-bit images (PNG/JPEG/BMP... decoded to RGBA8 sRGB, EImageDataType::Byte), perspective and
OpenCV / OpenCV-fisheye lenses, per-frame intrinsics overrides, `scale` / `offset` / `aabb` /
`aabb_scale`, the sharpness filter, `n_frames`, `white_transparent` / `black_transparent`,
`<file>.alpha.<ext>` alpha images and `dynamic_mask_<name>.png` masks. Not handled (the loader
raises): EXR/HDR images, depth supervision, per-pixel ray files, rolling shutter, FTheta / LatLong /
equirectangular lenses, Mitsuba scenes — none of the in-scope datasets use them.
Image decoding is PIL's (the reference uses stb_image); the pixels then travel to the device
unchanged, as `set_training_image` does with `convert_rgba32` (nerf_loader.cu:49-71).
"""
import json
import math
import os
import re

import numpy as np

from .nerf import LENS_OPENCV, LENS_OPENCV_FISHEYE, LENS_PERSPECTIVE, NerfDataset, make_image, nerf_matrix_to_ngp

NERF_SCALE = 0.33  # nerf_loader.h:29
IMAGE_FORMATS = ("png", "jpg", "jpeg", "bmp", "gif", "tga", "pic", "pnm", "psd", "exr")  # nerf_loader.cu:303-305
MASK_COLOR = 0x00FF00FF  # hot pink (nerf_loader.cu:580)


def _natural_key(s):
    """SI::natural::compare order (nerf_loader.cu:339-341): digit runs compare as numbers."""
    return [(0, int(t), "") if t.isdigit() else (1, 0, t) for t in re.split(r"(\d+)", s) if t != ""]


def _resolve(base, local):
    """resolve_path (nerf_loader.cu:307-318): try the known extensions when none is given."""
    path = local if os.path.isabs(local) else os.path.join(base, local)
    if not os.path.splitext(path)[1] and not os.path.exists(path):
        for ext in IMAGE_FORMATS:
            if os.path.exists(path + "." + ext):
                return path + "." + ext
    return path


def _load_json(path):
    with open(path, "r") as f:
        text = f.read()
    # nlohmann::json::parse(..., ignore_comments = true): strip // and /* */ comments outside strings
    out, i, n, in_str = [], 0, len(text), False
    while i < n:
        c = text[i]
        if in_str:
            out.append(c)
            if c == "\\" and i + 1 < n:
                out.append(text[i + 1])
                i += 1
            elif c == '"':
                in_str = False
        elif c == '"':
            in_str = True
            out.append(c)
        elif text.startswith("//", i):
            while i < n and text[i] != "\n":
                i += 1
            continue
        elif text.startswith("/*", i):
            j = text.find("*/", i + 2)
            i = n if j < 0 else j + 2
            continue
        else:
            out.append(c)
        i += 1
    return json.loads("".join(out))


def _read_lens(j, lens):
    """read_lens (nerf_loader.cu:160-224) into lens = {mode, params[4], principal[2]}."""
    opencv_mode = LENS_OPENCV_FISHEYE if j.get("is_fisheye", False) else LENS_OPENCV
    mode = LENS_PERSPECTIVE
    for name, idx in (("k1", 0), ("k2", 1), ("k3", 2), ("k4", 3), ("p1", 2), ("p2", 3)):
        if name in j:
            lens["params"][idx] = float(j[name])
            if lens["params"][idx] != 0.0:
                mode = opencv_mode
    if "cx" in j:
        lens["principal"][0] = float(np.float32(j["cx"]) / np.float32(j["w"]))
    if "cy" in j:
        lens["principal"][1] = float(np.float32(j["cy"]) / np.float32(j["h"]))
    if "rolling_shutter" in j:
        raise NotImplementedError("rolling_shutter datasets are not supported by this loader")
    for k in ("ftheta_p0", "latlong", "equirectangular"):
        if k in j:
            raise NotImplementedError(f"lens '{k}' is not supported (perspective / OpenCV / OpenCV fisheye only)")
    if mode != LENS_PERSPECTIVE:
        lens["mode"] = mode


def _fov_to_focal(res, degrees):
    """fov_to_focal_length (common.h), float arithmetic."""
    f32 = np.float32
    return float(f32(0.5) * f32(res) / np.tan(f32(0.5) * f32(degrees) * f32(math.pi) / f32(180)))


def _read_focal(j, res):
    """read_focal_length (nerf_loader.cu:226-258); returns (fx, fy) or None."""
    def axis(r, a):
        if a + "_fov" in j:
            return _fov_to_focal(r, j[a + "_fov"])
        if "fl_" + a in j:
            return float(np.float32(j["fl_" + a]))
        if "camera_angle_" + a in j:
            return _fov_to_focal(r, np.float32(j["camera_angle_" + a]) * np.float32(180) / np.float32(math.pi))
        return 0.0
    x, y = axis(res[0], "x"), axis(res[1], "y")
    if x != 0.0:
        return (x, y if y != 0.0 else x)
    if y != 0.0:
        return (y, y)
    return None


def _decode(path):
    from PIL import Image  # image decoding only (the reference uses stb_image)
    with Image.open(path) as im:
        return np.array(im.convert("RGBA"), dtype=np.uint8)


def _srgb_to_linear(x):
    return np.where(x <= 0.04045, x / 12.92, ((x + 0.055) / 1.055) ** 2.4)


class LoadedNerf:
    """Result of load_nerf: cameras + RGBA8 pixels (host) and the dataset-level settings."""

    def __init__(self):
        self.images, self.rgba8, self.paths = [], [], []
        self.scale, self.offset, self.aabb_scale = NERF_SCALE, [0.5, 0.5, 0.5], 1.0
        self.up = [0.0, 1.0, 0.0]

    def __len__(self):
        return len(self.images)

    def to_device(self):
        """NerfDataset (pixels and cameras uploaded: set_training_image)."""
        return NerfDataset(self.images, self.rgba8)


def load_nerf(jsonpaths, max_images=None):
    """load_nerf (nerf_loader.cu:260-726). jsonpaths: a transforms.json, a directory holding
    transforms*.json, or a list of json files."""
    if isinstance(jsonpaths, (str, os.PathLike)):
        p = os.fspath(jsonpaths)
        if os.path.isdir(p):
            jsonpaths = sorted(os.path.join(p, f) for f in os.listdir(p) if f.startswith("transforms") and f.endswith(".json"))
        else:
            jsonpaths = [p]
    if not jsonpaths:
        raise ValueError("Cannot load NeRF data from an empty set of paths.")
    res = LoadedNerf()
    jsons = [_load_json(p) for p in jsonpaths]
    per_json_frames = []
    for path, j in zip(jsonpaths, jsons):
        base = os.path.dirname(path)
        if not isinstance(j.get("frames"), list):
            per_json_frames.append([])
            continue
        frames = sorted(j["frames"], key=lambda fr: _natural_key(fr["file_path"]))
        for fr in frames:
            fr["file_path"] = fr["file_path"].replace("\\", "/")
        if "n_frames" in j:
            frames = frames[:min(len(frames), int(j["n_frames"]))]
        thresh = float(j.get("sharpness_discard_threshold", 0.0))
        if frames and "sharpness" in frames[0]:
            # kill frames blurrier than their neighbours (:349-372); also drops missing files
            kept = []
            for i in range(len(frames)):
                s0, s1 = max(0, i - 3), min(i + 3, len(frames) - 1)
                mean = sum(float(frames[k].get("sharpness", 1.0)) for k in range(s0, s1))
                mean = mean / (s1 - s0) if s1 > s0 else float("nan")
                if os.path.exists(_resolve(base, frames[i]["file_path"])) and float(frames[i].get("sharpness", 1.0)) > thresh * mean:
                    kept.append(frames[i])
            frames = kept
        per_json_frames.append(frames)
    for path, j, frames in zip(jsonpaths, jsons, per_json_frames):
        base = os.path.dirname(path)
        if j.get("normal_mts_args") is not None:
            raise NotImplementedError("Mitsuba scenes are not supported")
        if "camera" in j and isinstance(j["camera"], list):
            raise ValueError("hdf5 is no longer supported. please use the hdf52nerf.py conversion script")
        white = bool(j.get("white_transparent", False))
        black = bool(j.get("black_transparent", False))
        if "scale" in j:
            res.scale = float(j["scale"])
        if "aabb_scale" in j:
            res.aabb_scale = float(j["aabb_scale"])
        if "offset" in j:
            o = j["offset"]
            res.offset = [float(v) for v in o] if isinstance(o, list) else [float(o)] * 3
        if "aabb" in j:
            a = j["aabb"]
            length = max(1e-6, max(abs(float(a[1][k]) - float(a[0][k])) for k in range(3)))
            res.scale = 1.0 / length
            res.offset = [(float(a[1][k]) + float(a[0][k])) * 0.5 * -res.scale + 0.5 for k in range(3)]
        if "up" in j:
            res.up = [float(j["up"][1]), float(j["up"][2]), float(j["up"][0])]
        if "integer_depth_scale" in j or any("depth_path" in fr for fr in frames):
            pass  # depth supervision is not part of the training path here: ignored like a missing depth file
        lens0 = {"mode": LENS_PERSPECTIVE, "params": [0.0] * 4, "principal": [0.5, 0.5]}
        _read_lens(j, lens0)
        for fr in frames:
            if max_images is not None and len(res.images) >= max_images:
                break
            p = _resolve(base, fr["file_path"] or "")
            if not os.path.exists(p):
                raise FileNotFoundError(f"Could not find image file '{p}'.")
            if p.lower().endswith(".exr"):
                raise NotImplementedError("EXR (HDR) training images are not supported")
            px = _decode(p)
            h, w = px.shape[:2]
            ap = _resolve(base, f"{fr['file_path']}.alpha.{os.path.splitext(p)[1]}")
            if os.path.exists(ap):
                a = _decode(ap)
                if a.shape[:2] != (h, w):
                    raise ValueError(f"Alpha image {ap} has wrong resolution.")
                px[..., 3] = (255.0 * _srgb_to_linear(a[..., 0].astype(np.float32) / 255.0)).astype(np.uint8)
            mp = os.path.join(os.path.dirname(p), f"dynamic_mask_{os.path.splitext(os.path.basename(p))[0]}.png")
            mask_color = 0
            if os.path.exists(mp):
                m = _decode(mp)
                if m.shape[:2] != (h, w):
                    raise ValueError(f"Dynamic mask {mp} has wrong resolution.")
                mask_color = MASK_COLOR
                px.view(np.uint32)[..., 0][np.any(m[..., :3] != 0, axis=-1)] = MASK_COLOR
            # convert_rgba32 (nerf_loader.cu:49-71)
            if white:
                px[..., 3][np.all(px[..., :3] == 255, axis=-1)] = 0
            if black:
                px[..., 3][np.all(px[..., :3] == 0, axis=-1)] = 0
            if mask_color:
                px.view(np.uint32)[..., 0][px.view(np.uint32)[..., 0] == mask_color] = 0x00FF00FF
            focal = _read_focal(fr, (w, h)) or _read_focal(j, (w, h))
            if focal is None:
                raise ValueError("Couldn't read fov.")
            if "transform_matrix_end" in fr and fr.get("transform_matrix_end") != fr.get("transform_matrix_start", fr.get("transform_matrix")):
                pass  # only the start transform is used without a rolling shutter (t = 0)
            mat = fr.get("transform_matrix_start", fr["transform_matrix"])
            lens = {"mode": lens0["mode"], "params": list(lens0["params"]), "principal": list(lens0["principal"])}
            _read_lens(fr, lens)  # per-frame override (:676)
            xf = nerf_matrix_to_ngp(np.asarray(mat, np.float32), res.scale, res.offset)
            res.images.append(make_image(w, h, xf, focal=focal, principal=lens["principal"], lens_mode=lens["mode"],
                                         lens_params=lens["params"]))
            res.rgba8.append(px)
            res.paths.append(p)
    if not res.images:
        raise ValueError("No training images were found for NeRF training!")
    return res
