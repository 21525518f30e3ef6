"""Minimal FITS primary-array reader/writer.

The reference reads and writes its images with astropy.io.fits
(application_sgp_subdivisions.py:25-60, sgp.py:218-236 ``save``; data files
results/*.fits, psf/*_img.fits): simple primary HDUs, BITPIX -32/-64 (and
integer BITPIX with BSCALE/BZERO in general), big-endian samples.  This module
parses the 2880-byte header blocks itself and hands the raw data block to the
device, where ``bsgp_fits_to_f64`` byte-swaps and widens it (one H2D copy of
the file's bytes, no host-side decode), so batches stream without astropy.

  read_fits(path)            -> (header dict, numpy array, file dtype, native order)
  read_fits_device(path)     -> (header dict, float64 CUDA tensor [NAXIS2, NAXIS1])
  write_fits(path, array)    -> primary HDU with the cards astropy writes for a
                                plain array (byte-identical to the reference's files)
"""
import os

import numpy as np

import _bsgp as _B

BLOCK = 2880
_DTYPE = {8: ">u1", 16: ">i2", 32: ">i4", 64: ">i8", -32: ">f4", -64: ">f8"}
_BITPIX = {np.dtype(np.uint8): 8, np.dtype(np.int16): 16, np.dtype(np.int32): 32,
           np.dtype(np.int64): 64, np.dtype(np.float32): -32, np.dtype(np.float64): -64}


class FitsError(ValueError):
    pass


def _value(v):
    v = v.strip()
    if v.startswith("'"):
        return v[1:v.rfind("'")].rstrip()
    if v in ("T", "F"):
        return v == "T"
    try:
        return int(v)
    except ValueError:
        try:
            return float(v.replace("D", "E"))
        except ValueError:
            return v


def read_header(f):
    """Cards of the primary header up to END; returns (dict, data offset)."""
    hdr = {}
    nblk = 0
    while True:
        blk = f.read(BLOCK)
        if len(blk) < BLOCK:
            raise FitsError("truncated FITS header")
        nblk += 1
        for i in range(0, BLOCK, 80):
            card = blk[i:i + 80].decode("ascii", "replace")
            key = card[:8].strip()
            if key == "END":
                if "SIMPLE" not in hdr or not hdr["SIMPLE"]:
                    raise FitsError("not a simple FITS file")
                return hdr, nblk * BLOCK
            if card[8:10] == "= ":
                val = card[10:]
                if not val.lstrip().startswith("'") and "/" in val:
                    val = val[:val.index("/")]
                hdr[key] = _value(val)


def _geometry(hdr):
    bitpix = int(hdr["BITPIX"])
    if bitpix not in _DTYPE:
        raise FitsError(f"unsupported BITPIX {bitpix}")
    naxis = int(hdr.get("NAXIS", 0))
    shape = tuple(int(hdr[f"NAXIS{i}"]) for i in range(naxis, 0, -1))  # C order
    n = int(np.prod(shape)) if naxis else 0
    return bitpix, shape, n


def read_fits(path):
    """Primary array as numpy in the file's sample type (native byte order),
    with BSCALE/BZERO applied (as astropy does) when present."""
    with open(path, "rb") as f:
        hdr, off = read_header(f)
        bitpix, shape, n = _geometry(hdr)
        raw = f.read(n * abs(bitpix) // 8)
    if len(raw) < n * abs(bitpix) // 8:
        raise FitsError("truncated FITS data")
    data = np.frombuffer(raw, dtype=_DTYPE[bitpix]).reshape(shape)
    bscale, bzero = float(hdr.get("BSCALE", 1.0)), float(hdr.get("BZERO", 0.0))
    if bscale != 1.0 or bzero != 0.0:
        return hdr, bzero + bscale * data.astype(np.float64)
    return hdr, data.astype(data.dtype.newbyteorder("="))


def read_fits_device(path):
    """Primary array as a float64 CUDA tensor: the raw data block is copied to
    the device as is and decoded there (bsgp_fits_to_f64)."""
    _B.require_gpu()
    torch = _B.torch
    with open(path, "rb") as f:
        hdr, off = read_header(f)
        bitpix, shape, n = _geometry(hdr)
        nbytes = n * abs(bitpix) // 8
        raw = np.fromfile(f, dtype=np.uint8, count=nbytes)
    if raw.size < nbytes:
        raise FitsError("truncated FITS data")
    dev = torch.from_numpy(raw).to("cuda")
    out = torch.empty(shape, dtype=torch.float64, device="cuda")
    _B.check(_B.lib().bsgp_fits_to_f64(_B._ptr(dev), n, bitpix, float(hdr.get("BSCALE", 1.0)),
                                       float(hdr.get("BZERO", 0.0)), _B._ptr(out),
                                       _B.current_stream()))
    out._keep = dev  # the raw block lives until the decode ran
    return hdr, out


def _card(key, value=None, comment=None):
    if value is None:
        c = f"{key:<8}"
    else:
        v = "T" if value is True else ("F" if value is False else str(value))
        c = f"{key:<8}= {v:>20}"
        if comment:
            c += f" / {comment}"
    return c.ljust(80)[:80]


def write_fits(path, data, overwrite=False):
    """Primary HDU of a 1-3-D array with the cards astropy writes for a plain
    array (SIMPLE, BITPIX, NAXIS, NAXISn, EXTEND, END), big-endian samples,
    both parts zero/space-padded to 2880-byte blocks."""
    if os.path.exists(path) and not overwrite:
        raise FitsError(f"{path} exists")
    data = np.asarray(data)
    if data.dtype not in _BITPIX:
        raise FitsError(f"unsupported dtype {data.dtype}")
    bitpix = _BITPIX[data.dtype]
    cards = [_card("SIMPLE", True, "conforms to FITS standard"),
             _card("BITPIX", bitpix, "array data type"),
             _card("NAXIS", data.ndim, "number of array dimensions")]
    for i, n in enumerate(reversed(data.shape)):
        cards.append(_card(f"NAXIS{i + 1}", n))
    cards.append(_card("EXTEND", True))
    cards.append("END".ljust(80))
    head = "".join(cards).encode("ascii")
    head += b" " * (-len(head) % BLOCK)
    body = np.ascontiguousarray(data).astype(_DTYPE[bitpix]).tobytes()
    body += b"\0" * (-len(body) % BLOCK)
    with open(path, "wb") as f:
        f.write(head)
        f.write(body)
