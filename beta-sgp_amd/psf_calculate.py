"""DIAPL PSF model on the device: drop-in for psf/psf_calculate.py's ``PSF``
(SURVEY §8f row 4).

Same attributes and methods as the reference class (psf_calculate.py:9-165);
the stamps are computed by ``bsgp_psf_stamps`` on the GPU.  Two additions
serve the subdivision pipeline:

  psf.stamps(xy, normalize=True, device_out=False)
      one stamp per field position (x, y) through the model's spatial
      expansion (what init_psf, :140-165, sets out to do), as [n, S, S];
  psf.local_coeffs(x, y)
      the local coefficient vector at (x, y) — init_psf's result (the
      reference's version raises TypeError and returns nothing).

Stamps are (2hw+1)^2 with pixel (r, c) = calc_psf_pix(x = c - hw, y = r - hw),
exactly get_psf_mat's 31x31 layout for the hw = 15 of DIAPL's PSFHW.
"""
import numpy as np

import _bsgp as _B


class PSF:
    def __init__(self, txt_file):
        """Read a DIAPL coefficient file (psf_calculate.py:10-47)."""
        self.ldeg = 2
        self.sdeg = 1
        with open(txt_file) as f:
            data = [float(l.rstrip("\n")) for l in f]
        self.hw = int(data[0])
        self.ndeg_spat = int(data[1])
        self.ndeg_local = int(data[2])
        self.ngauss = int(data[3])
        self.recenter = data[4]
        self.cos = data[5]
        self.sin = data[6]
        self.ax = data[7]
        self.ay = data[8]
        self.sigma_inc = data[9]
        self.sigma_mscale = data[10]
        self.fitrad = data[11]
        self.x_orig = data[12]
        self.y_orig = data[13]
        self.vec_coeffs = data[14:]
        self.ntot = self.ngauss * (self.ndeg_local + 1) * (self.ndeg_local + 2) / 2
        self.ntot *= (self.ndeg_spat + 1) * (self.ndeg_spat + 2) / 2

    @property
    def coeffs(self):
        return self.vec_coeffs

    @property
    def ncomp(self):
        return self.ngauss * (self.ldeg + 1) * (self.ldeg + 2) // 2

    # ----------------------------------------------------------- device
    def _model(self, hw=None):
        c = np.ascontiguousarray(self.vec_coeffs, dtype=np.float64)
        m = _B.PsfModel(hw=self.hw if hw is None else hw, ngauss=self.ngauss, ldeg=self.ldeg,
                        sdeg=self.sdeg, cos=self.cos, sin=self.sin, ax=self.ax, ay=self.ay,
                        sigma_inc=self.sigma_inc, x_orig=self.x_orig, y_orig=self.y_orig,
                        coeffs=c.ctypes.data, ncoef=len(c))
        return m, c

    def _stamps(self, xy, n, normalize, hw=None):
        _B.require_gpu()
        torch = _B.torch
        m, keep = self._model(hw)
        S = 2 * m.hw + 1
        out = torch.empty((n, S, S), dtype=torch.float64, device="cuda")
        _B.check(_B.lib().bsgp_psf_stamps(_B.ctypes.byref(m), _B._ptr(xy) if xy is not None else None,
                                          n, int(xy is not None), int(bool(normalize)),
                                          _B._ptr(out), _B.current_stream()))
        del keep  # the coefficients are copied into the kernel arguments at launch
        return out

    def stamps(self, xy, normalize=True, device_out=False):
        """Stamps at field positions xy [n, 2] ((x, y) pairs): the local
        coefficients come from the spatial expansion about (x_orig, y_orig)."""
        torch = _B.torch
        _B.require_gpu()
        xy_d = xy.to(dtype=torch.float64).contiguous() if torch.is_tensor(xy) else \
            _B.to_dev(np.asarray(xy, dtype=np.float64).reshape(-1, 2))
        out = self._stamps(xy_d, xy_d.shape[0], normalize)
        out._keep = xy_d
        if device_out:
            return out
        return out.cpu().numpy()

    def local_coeffs(self, x, y):
        """init_psf (:140-165): local coefficients at field position (x, y)."""
        ncomp = self.ncomp
        loc = [0.0] * ncomp
        itot = 0
        a1 = 1.0
        for m in range(self.sdeg + 1):
            a2 = 1.0
            for _ in range(self.sdeg - m + 1):
                for icomp in range(ncomp):
                    loc[icomp] += self.vec_coeffs[itot] * a1 * a2
                    itot += 1
                a2 *= y - self.y_orig
            a1 *= x - self.x_orig
        return loc

    def init_psf(self, xpsf, ypsf):
        """The reference's init_psf, returning the local coefficient vector."""
        return self.local_coeffs(xpsf, ypsf)

    # ------------------------------------------------------ reference API
    def calc_psf_pix(self, coeffs, x, y):
        """PSF value at integer pixel offset (x, y) (psf_calculate.py:52-87).
        As in the reference, the value uses the model's own coefficients
        (``coeffs`` is not read there either)."""
        if int(x) != x or int(y) != y:
            raise ValueError("calc_psf_pix evaluates integer pixel offsets")
        hw = max(abs(int(x)), abs(int(y)))
        st = self._stamps(None, 1, False, hw=hw)[0]
        return float(st[int(y) + hw, int(x) + hw])

    def get_psf_mat(self):
        """(2hw+1)^2 stamp at the expansion origin (psf_calculate.py:89-107)."""
        self.psf_mat = self._stamps(None, 1, False)[0].cpu().numpy()
        return self.psf_mat

    def show_psf_mat(self):
        import matplotlib.pyplot as plt  # display only (psf_calculate.py:109-114)
        plt.matshow(self.get_psf_mat(), origin='lower')
        plt.colorbar()
        plt.show()

    def check_symmetric(self, coeffs, rtol=1e-05, atol=1e-08):
        return np.allclose(coeffs, coeffs.T, rtol=rtol, atol=atol)

    def normalize_psf_mat(self):
        """Stamp divided by its sum (psf_calculate.py:129-137)."""
        self.get_psf_mat()
        return self._stamps(None, 1, True)[0].cpu().numpy()
