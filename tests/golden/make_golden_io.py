"""Golden fixtures for the data paths either side of the solver (SURVEY §8f
rows 2-3), generated from the REFERENCE and astropy in the build container:

    cd /root/repo && PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 tests/golden/make_golden_io.py

* ``ref_slice_bboxes.npz``: restoration/utils.py:332-372 ``calculate_slice_bboxes``
  on a grid of (field, tile, overlap) cases, including the ones where
  ``int(overlap/size*size)`` rounds down; the function is taken from the
  reference's source text (``ast``) and executed alone, because utils.py's
  module imports (sep, photutils, reproject, ndpatch, ...) are absent here.
* ``ref_cutouts.npz``: astropy 4.3.1 ``Cutout2D`` (utils.py:383) of a random
  field at the centres/sizes ``create_subdivisions`` uses.
* ``ref_fits_io.npz`` + two FITS files copied from the reference
  (psf/psfccfbrd210048_1_1_img.fits, BITPIX -64; results/SUBDIV_ORIGIMG.fits,
  BITPIX -32): astropy's decoded arrays as sha256 of their native-f64 bytes,
  shape and a few values.
"""
import ast
import hashlib
import os
import shutil

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def reference_function(path, name):
    src = open(path).read()
    tree = ast.parse(src)
    node = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name)
    ns = {}
    exec(compile(ast.Module(body=[node], type_ignores=[]), path, "exec"), ns)
    return ns[name]


def main():
    bboxes = reference_function(os.path.join(REF, "restoration", "utils.py"),
                                "calculate_slice_bboxes")
    cases = [(375, 375, 100, 100, 10), (2048, 2048, 256, 256, 32), (1024, 768, 256, 256, 29),
             (300, 500, 128, 96, 17), (256, 256, 256, 256, 0), (1000, 1000, 300, 300, 57),
             (4100, 4100, 512, 512, 64), (513, 1025, 256, 256, 1),
             (600, 700, 100, 100, 29), (900, 900, 300, 300, 55)]  # int(ov/s*s) == ov - 1
    out = {}
    for i, (H, W, sh, sw, ov) in enumerate(cases):
        # create_subdivisions passes overlap/size as the ratio (utils.py:378-381)
        b = np.array(bboxes(H, W, sh, sw, ov / sh, ov / sw), dtype=np.int32)
        out[f"case{i}"] = np.array([H, W, sh, sw, ov], dtype=np.int64)
        out[f"boxes{i}"] = b
    np.savez(os.path.join(OUT, "ref_slice_bboxes.npz"), **out)

    # astropy 4.3.1 on numpy 1.26 needs these removed numpy aliases (as make_golden.py)
    if not hasattr(np, "asscalar"):
        np.asscalar = lambda a: a.item()
    if not hasattr(np, "alen"):
        np.alen = len
    from astropy.nddata import Cutout2D
    rng = np.random.default_rng(3)
    img = rng.normal(100.0, 10.0, (150, 200))
    H, W, sh, sw, ov = 150, 200, 48, 40, 7
    b = np.array(bboxes(H, W, sh, sw, ov / sh, ov / sw), dtype=np.int32)
    cut = np.stack([Cutout2D(img, ((s[0] + s[2]) / 2, (s[1] + s[3]) / 2), size=(sh, sw)).data
                    for s in b])
    np.savez(os.path.join(OUT, "ref_cutouts.npz"), img=img, boxes=b, cutouts=cut,
             shape=np.array([sh, sw]))

    from astropy.io import fits
    res = {}
    for tag, rel in [("psf", "psf/psfccfbrd210048_1_1_img.fits"),
                     ("subdiv", "results/SUBDIV_ORIGIMG.fits")]:
        src = os.path.join(REF, rel)
        dst = os.path.join(OUT, os.path.basename(rel))
        shutil.copyfile(src, dst)
        with fits.open(src) as h:
            d = h[0].data
            res[f"{tag}_shape"] = np.array(d.shape)
            res[f"{tag}_bitpix"] = np.array(h[0].header["BITPIX"])
            nat = np.asarray(d, dtype=np.float64)
            res[f"{tag}_sha256"] = np.array(hashlib.sha256(nat.tobytes()).hexdigest())
            res[f"{tag}_sum"] = np.array(nat.sum())
            res[f"{tag}_row0"] = nat[0].copy()
            res[f"{tag}_file"] = np.array(os.path.basename(rel))
    np.savez(os.path.join(OUT, "ref_fits_io.npz"), **res)
    print("wrote ref_slice_bboxes.npz, ref_cutouts.npz, ref_fits_io.npz and the FITS files")


if __name__ == "__main__":
    main()
