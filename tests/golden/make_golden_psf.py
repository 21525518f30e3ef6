"""Golden fixtures for the DIAPL PSF model, generated from
the REFERENCE in the build container:

    cd /root/repo && PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 tests/golden/make_golden_psf.py

The reference's ``PSF`` class (psf/psf_calculate.py:9-165) is taken from its
source text (``ast``) and run alone (the module's matplotlib/astropy imports
are not needed by the class).  ``ref_psf_model.npz`` holds, for the
reference's coefficient file psf/psfccfbrd210048_1_1.bin.txt (copied here as
data) and for synthetic coefficient files (ngauss 1-3, rotations), the file's
values, ``get_psf_mat()`` and ``normalize_psf_mat()``.  The reference's own
normalised stamp of that file, psf/psfccfbrd210048_1_1_img.fits, is already a
fixture (make_golden_io.py).  ``init_psf`` (the spatial expansion) cannot run
in the reference (``[0.0] * ncomp`` with a float ncomp raises TypeError), so
spatial stamps have no reference vector: parity there is against the
restated formula only (unpinned).
"""
import ast
import os
import shutil

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def reference_class(path, name):
    tree = ast.parse(open(path).read())
    node = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == name)
    ns = {"np": np}
    exec(compile(ast.Module(body=[node], type_ignores=[]), path, "exec"), ns)
    return ns[name]


def synthetic(rng, ngauss, ndeg_spat=1, angle=0.3):
    ncomp = ngauss * 6
    nterm = (ndeg_spat + 1) * (ndeg_spat + 2) // 2
    coef = rng.normal(0, 1e-3, ncomp * nterm)
    coef[0] = 0.1  # dominant Gaussian term
    hdr = [15, ndeg_spat, 2, ngauss, 1, np.cos(angle), np.sin(angle), -rng.uniform(0.1, 0.3),
           -rng.uniform(0.1, 0.3), 0.548, 1.582, 3, 225, 225]
    return hdr + list(coef)


def main():
    PSF = reference_class(os.path.join(REF, "psf", "psf_calculate.py"), "PSF")
    src = os.path.join(REF, "psf", "psfccfbrd210048_1_1.bin.txt")
    shutil.copyfile(src, os.path.join(OUT, "psfccfbrd210048_1_1.bin.txt"))
    rng = np.random.default_rng(7)
    files = [src]
    for i, (ng, ang) in enumerate([(1, 0.0), (2, 0.7), (3, -1.2)]):
        p = f"/tmp/psf_synth{i}.bin.txt"
        with open(p, "w") as f:
            for v in synthetic(rng, ng, 1, ang):
                f.write(f"{float(v)!r}\n")
        files.append(p)
    out = {}
    for i, p in enumerate(files):
        psf = PSF(p)
        out[f"file{i}"] = np.array([float(l) for l in open(p)])
        out[f"raw{i}"] = psf.get_psf_mat()
        out[f"norm{i}"] = psf.normalize_psf_mat()
    np.savez(os.path.join(OUT, "ref_psf_model.npz"), **out)
    print("wrote ref_psf_model.npz and psfccfbrd210048_1_1.bin.txt")


if __name__ == "__main__":
    main()
