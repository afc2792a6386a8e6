"""Training-data loaders of the reference's TF workloads.

* :func:`load_csv` / :func:`open_text` — the health.csv MLP loader (train_tf_ps.py:53-149): keep
  rows with a non-empty label and all numeric features present and not NaN; sorted label
  vocabulary -> int32 labels; float32 features.  Parsing goes through the native CSV tokenizer.
* :func:`count_images` / :func:`make_image_dataset` — the laser-spot regression set
  (train_tf_ps.py:168-322): flat directory + ``clean_labels.jsonl`` with
  ``{"image", "point": {"x_px", "y_px"}}``; deterministic seeded split; decode -> resize ->
  batch.  Decoding is on the host (PIL); the bilinear resize + /255 + channel padding run on the
  GPU inside the first convolution op when images arrive at their native size, so only uint8
  pixels cross PCIe.
* :func:`write_synthetic_image_dataset` — generates a laser-spot-shaped dataset (the real
  ``laser-spots`` images are not in the reference repo, .gitignore:9).
"""
from __future__ import annotations

import io
import json
import os
from typing import List, Optional, Tuple

import numpy as np

from .dataset import AUTOTUNE, Dataset

IMAGE_EXTS = {".jpg", ".jpeg", ".png", ".bmp", ".gif", ".ppm"}


def open_text(path_or_url: str) -> io.TextIOBase:
    if path_or_url.startswith(("http://", "https://")):
        from urllib.request import urlopen

        return io.TextIOWrapper(urlopen(path_or_url), encoding="utf-8")
    return open(path_or_url, "r", encoding="utf-8")


def load_csv(source: str, numeric_features: Optional[List[str]] = None,
             label_col: str = "subpopulation") -> Tuple[np.ndarray, np.ndarray, List[str]]:
    from ..sql.readwriter import _parse_csv_bytes

    numeric_features = numeric_features or ["value", "lower_ci", "upper_ci"]
    if source.startswith(("http://", "https://")):
        with open_text(source) as fh:
            buf = fh.read().encode("utf-8")
    else:
        with open(source, "rb") as fh:
            buf = fh.read()
    t = _parse_csv_bytes(buf, header=True, infer=False, sep=",", device="cpu", rank_split=False)
    lab = t.column(label_col)
    labels = np.array([(s.strip() if s is not None else "") for s in (lab.dictionary or [])] + [""], dtype=object)
    codes = lab.data.numpy()
    lab_str = labels[np.where(codes >= 0, codes, len(labels) - 1)]
    keep = lab_str != ""
    feats = []
    for c in numeric_features:
        cv = t.column(c)
        d = cv.dictionary or []
        vals = np.empty(len(d) + 1, dtype=np.float64)
        for i, s in enumerate(d):
            s2 = s.strip()
            try:
                vals[i] = float(s2) if s2 and s2.lower() != "nan" else np.nan
            except ValueError:
                vals[i] = np.nan
        vals[-1] = np.nan
        cc = cv.data.numpy()
        x = vals[np.where(cc >= 0, cc, len(d))]
        keep &= ~np.isnan(x)
        feats.append(x)
    if not keep.any():
        raise RuntimeError("No valid rows were parsed from the dataset.")
    X = np.stack([f[keep] for f in feats], 1).astype(np.float32)
    ys = lab_str[keep]
    vocab = sorted(set(ys.tolist()))
    index = {s: i for i, s in enumerate(vocab)}
    y = np.array([index[s] for s in ys], dtype=np.int32)
    return X, y, vocab


def list_image_classes(data_dir: str):
    raise RuntimeError("Folder-per-class structure is no longer supported. Use clean_labels.jsonl with a flat "
                       "image directory.")


def _label_entries(data_dir: str):
    labels_path = os.path.join(data_dir, "clean_labels.jsonl")
    if not os.path.isfile(labels_path):
        raise RuntimeError(f"clean_labels.jsonl not found in: {data_dir}")
    out = []
    with open(labels_path, "r", encoding="utf-8") as fh:
        for line in fh:
            line = line.strip()
            if not line:
                continue
            try:
                obj = json.loads(line)
            except Exception:  # noqa: BLE001 - skip malformed lines like the reference
                continue
            name = str(obj.get("image", "")).strip()
            if not name or os.path.splitext(name.lower())[1] not in IMAGE_EXTS:
                continue
            full = os.path.join(data_dir, name)
            if not os.path.isfile(full):
                continue
            pt = obj.get("point") or {}
            out.append((full, pt.get("x_px"), pt.get("y_px")))
    return out


def count_images(data_dir: str) -> int:
    n = len(_label_entries(data_dir))
    if n == 0:
        raise RuntimeError("No labeled images found (clean_labels.jsonl present but matched zero files).")
    return n


def _decode(path: str, h: int, w: int) -> np.ndarray:
    from PIL import Image

    with Image.open(path) as im:
        im = im.convert("RGB")
        if im.size != (w, h):
            im = im.resize((w, h), Image.BILINEAR)
        return np.asarray(im, dtype=np.uint8)


def make_image_dataset(data_dir: str, image_size, batch_size: int, shuffle: bool = True, input_context=None,
                       validation_split: float = 0.0, subset: Optional[str] = None, seed: int = 1337,
                       repeat: bool = True, cache: bool = False) -> Dataset:
    """``cache=True``: decode once into an HBM-resident uint8 tensor and serve batches by device
    gathers (see _resident_image_dataset); otherwise the reference's streaming pipeline
    (train_tf_ps.py:297-321: decode map -> shuffle(3000) -> batch -> repeat -> prefetch)."""
    img_h, img_w = int(image_size[0]), int(image_size[1])
    entries = [(p, x, y) for p, x, y in _label_entries(data_dir) if x is not None and y is not None]
    if not entries:
        raise RuntimeError("No valid labeled images were parsed from clean_labels.jsonl")
    idx = np.arange(len(entries))
    np.random.default_rng(seed).shuffle(idx)
    if validation_split and subset in ("training", "validation"):
        val = max(1, min(len(idx) - 1, int(len(idx) * float(validation_split))))
        idx = idx[:-val] if subset == "training" else idx[-val:]
    paths = [entries[i][0] for i in idx]
    targets = np.array([[entries[i][1], entries[i][2]] for i in idx], dtype=np.float32)
    if cache:
        return _resident_image_dataset(paths, targets, img_h, img_w, batch_size, shuffle, input_context, seed, repeat)
    ds = Dataset.zip((Dataset.from_tensor_slices(np.array(paths, dtype=object)), Dataset.from_tensor_slices(targets)))
    if input_context is not None:  # shard before decoding: each worker decodes only its own files
        ds = ds.shard(input_context.num_input_pipelines, input_context.input_pipeline_id)
    ds = ds.map(lambda p, y: (_decode(str(p), img_h, img_w), y), num_parallel_calls=AUTOTUNE)
    if shuffle:
        ds = ds.shuffle(min(3000, len(paths)), seed=seed)
    ds = ds.batch(batch_size)
    if repeat:
        ds = ds.repeat()
    return ds.prefetch(1)


def _resident_image_dataset(paths, targets, img_h, img_w, batch_size, shuffle, input_context, seed, repeat):
    """Decode this worker's images ONCE (thread pool; PIL releases the GIL while decoding) into one
    uint8 [N, H, W, 3] array kept resident in HBM (a laser-spot set of a few thousand 256x320 frames
    is ~1 GB of the GPU's 288 GB), then shuffle / batch / repeat as a columnar plan: every batch is
    an index gather on the device, so the host never touches pixels again after the first pass."""
    import concurrent.futures as cf

    import torch

    sel = np.arange(len(paths))
    if input_context is not None:
        sel = sel[input_context.input_pipeline_id::input_context.num_input_pipelines]
    imgs = np.empty((len(sel), img_h, img_w, 3), dtype=np.uint8)

    def dec(j):
        imgs[j] = _decode(str(paths[sel[j]]), img_h, img_w)

    with cf.ThreadPoolExecutor(max(4, min(16, os.cpu_count() or 4))) as ex:
        list(ex.map(dec, range(len(sel))))
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    x = torch.from_numpy(imgs).to(dev)
    y = torch.from_numpy(targets[sel]).to(dev)
    ds = Dataset.from_tensor_slices((x, y))
    if shuffle:
        ds = ds.shuffle(len(sel), seed=seed)
    ds = ds.batch(batch_size)
    if repeat:
        ds = ds.repeat()
    return ds


def synthetic_laser_spots(n: int, size=(256, 320), seed: int = 0):
    """Yield ``n`` (uint8 [H, W, 3] frame, (x_px, y_px)) laser-spot-like samples: a dark noisy frame
    with one bright red Gaussian spot (sigma 3 px) at a uniform random position >= 10 px from the
    border - the shape of the reference's laser-spot dataset (clean_labels.jsonl, train_tf_ps.py:
    234-268), which is not shipped with it."""
    rng = np.random.default_rng(seed)
    h, w = size
    yy, xx = np.mgrid[0:h, 0:w]
    for _ in range(n):
        x, y = float(rng.uniform(10, w - 10)), float(rng.uniform(10, h - 10))
        img = rng.integers(0, 40, (h, w, 3), dtype=np.uint8)
        spot = np.exp(-((xx - x) ** 2 + (yy - y) ** 2) / 18.0)
        img[..., 0] = np.clip(img[..., 0] + 215 * spot, 0, 255).astype(np.uint8)
        yield img, (x, y)


def write_synthetic_image_dataset(out_dir: str, n: int = 64, size=(256, 320), seed: int = 0) -> str:
    """A laser-spot-like dataset on disk (PNG frames + clean_labels.jsonl): :func:`synthetic_laser_spots`."""
    from PIL import Image

    os.makedirs(out_dir, exist_ok=True)
    h, w = size
    with open(os.path.join(out_dir, "clean_labels.jsonl"), "w") as fh:
        for i, (img, (x, y)) in enumerate(synthetic_laser_spots(n, size, seed)):
            name = f"img_{i:05d}.png"
            Image.fromarray(img).save(os.path.join(out_dir, name))
            fh.write(json.dumps({"image": name, "point": {"x_px": x, "y_px": y},
                                 "image_size": {"width": w, "height": h}}) + "\n")
    return out_dir
