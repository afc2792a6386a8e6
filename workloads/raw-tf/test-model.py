"""Manual model check: predict the laser-spot position on every image and save an annotated copy
(reference: workloads/raw-tf/test-model.py:13-56, ``ManualImageChecker``).

Loads ``<model-dir>/150-320-by-256-B1-model.keras`` (or ``--model``), resizes each PNG/JPEG to
320x256, scales by 1/255, predicts (x, y) with the forward-only path on the MI355X (or CPU) and writes
``<model-dir>/plots/<name>`` with a red marker at the prediction.  Plotting uses PIL (matplotlib is
not part of this runtime); ``--sleep`` keeps the reference's 1 s pause between images (default 0).
"""
import argparse
import glob
import os
import time

import _path  # noqa: F401
import numpy as np
from PIL import Image, ImageDraw

from pyspark_tf_gke_amd.nn.model import load_model

IMG_W, IMG_H = 320, 256


class ManualImageChecker:
    def __init__(self, model_path, plots_dir, device=None):
        self.model = load_model(model_path, device=device)
        self.model.summary()
        self.plots_dir = plots_dir
        os.makedirs(plots_dir, exist_ok=True)

    def predict(self, path):
        img = Image.open(path).convert("RGB").resize((IMG_W, IMG_H), Image.BILINEAR)
        x = np.asarray(img, dtype=np.float32)[None] / 255.0
        pred = np.asarray(self.model.predict(x, verbose=0))
        return float(pred[0, 0]), float(pred[0, 1]), img

    def plot(self, img, x, y, name):
        d = ImageDraw.Draw(img)
        r = 5
        d.ellipse([x - r, y - r, x + r, y + r], outline=(255, 0, 0), width=2)
        d.line([x - 2 * r, y, x + 2 * r, y], fill=(255, 0, 0))
        d.line([x, y - 2 * r, x, y + 2 * r], fill=(255, 0, 0))
        out = os.path.join(self.plots_dir, name)
        img.save(out)
        return out

    def run(self, image_dir, sleep=0.0):
        files = sorted(f for ext in ("*.png", "*.jpg", "*.jpeg") for f in glob.glob(os.path.join(image_dir, ext)))
        results = []
        for f in files:
            x, y, img = self.predict(f)
            out = self.plot(img, x, y, os.path.basename(f))
            print(f"{os.path.basename(f)}: predicted (x={x:.1f}, y={y:.1f}) -> {out}", flush=True)
            results.append((f, x, y))
            if sleep:
                time.sleep(sleep)
        return results


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model-dir", default="./tf-model")
    ap.add_argument("--model", default=None)
    ap.add_argument("--images", default="./images")
    ap.add_argument("--sleep", type=float, default=0.0)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    model = a.model or os.path.join(a.model_dir, "150-320-by-256-B1-model.keras")
    ManualImageChecker(model, os.path.join(a.model_dir, "plots"), a.device).run(a.images, a.sleep)


if __name__ == "__main__":
    main()
