"""Subdivision tiling and mosaic on the device.

The reference's application (application_sgp_subdivisions.py with
restoration/utils.py:332-395) cuts a field into overlapping subdivisions
(``calculate_slice_bboxes`` + astropy ``Cutout2D``), deconvolves each one with
``sgp_betaDiv`` and rebuilds the field with ``reproject_and_coadd``.  Here the
whole chain stays in HBM:

  boxes = calculate_slice_bboxes(...)           # utils.py:332-372, same boxes
  tiles = extract_tiles(field, boxes, shape)    # bsgp_extract_tiles  [n, th, tw]
  out   = sgp.sgp_betaDiv_batch(tiles, ...)     # one batched solve (one workgroup per tile)
  mosaic, footprint = coadd_tiles(out, boxes)   # bsgp_coadd_tiles, mean in tile order

``sgp_subdivisions`` runs the chain.  The co-add is the same-WCS case of
reproject_and_coadd with combine_function='mean'; its ``match_background``
offset fit (utils.py:391) is not reproduced (parity of that step is unpinned:
the reproject package is absent here).
"""
import numpy as np

import _bsgp as _B


def calculate_slice_bboxes(image_height, image_width, slice_height=512, slice_width=512,
                           overlap_height_ratio=0.2, overlap_width_ratio=0.2):
    """utils.py:332-372 (same boxes, xyxy, row-major; overlaps int(ratio*size))."""
    boxes = []
    y_max = y_min = 0
    y_overlap = int(overlap_height_ratio * slice_height)
    x_overlap = int(overlap_width_ratio * slice_width)
    while y_max < image_height:
        x_min = x_max = 0
        y_max = y_min + slice_height
        while x_max < image_width:
            x_max = x_min + slice_width
            if y_max > image_height or x_max > image_width:
                xmax = min(image_width, x_max)
                ymax = min(image_height, y_max)
                boxes.append([max(0, xmax - slice_width), max(0, ymax - slice_height), xmax, ymax])
            else:
                boxes.append([x_min, y_min, x_max, y_max])
            x_min = x_max - x_overlap
        y_min = y_max - y_overlap
    return boxes


def subdivision_boxes(shape, subdiv_shape=(100, 100), overlap=10):
    """The boxes create_subdivisions uses (utils.py:378-381: ratio = overlap/size)."""
    return np.asarray(calculate_slice_bboxes(shape[0], shape[1], subdiv_shape[0], subdiv_shape[1],
                                             overlap / subdiv_shape[0], overlap / subdiv_shape[1]),
                      dtype=np.int32)


def tile_centres(boxes):
    """(x, y) pixel centre of every box: ((x0 + x1 - 1) / 2, (y0 + y1 - 1) / 2)."""
    b = np.asarray(boxes, dtype=np.float64).reshape(-1, 4)
    return np.stack([(b[:, 0] + b[:, 2] - 1) / 2, (b[:, 1] + b[:, 3] - 1) / 2], axis=1)


def _field(image):
    torch = _B.torch
    if torch.is_tensor(image):
        return image.to(dtype=torch.float64).contiguous()
    return _B.to_dev(np.asarray(image, dtype=np.float64))


def extract_tiles(image, boxes, subdiv_shape):
    """[n, th, tw] float64 CUDA tensor of image[y0:y1, x0:x1] per box."""
    _B.require_gpu()
    torch = _B.torch
    img = _field(image)
    H, W = img.shape
    th, tw = subdiv_shape
    b = np.asarray(boxes, dtype=np.int32).reshape(-1, 4)
    if np.any(b[:, 2] - b[:, 0] != tw) or np.any(b[:, 3] - b[:, 1] != th) or \
            np.any(b[:, :2] < 0) or np.any(b[:, 2] > W) or np.any(b[:, 3] > H):
        raise ValueError("every box must be subdiv_shape sized and inside the field "
                         "(a field smaller than one subdivision yields smaller boxes)")
    bd = torch.from_numpy(np.ascontiguousarray(b)).to("cuda")
    out = torch.empty((len(b), th, tw), dtype=torch.float64, device="cuda")
    _B.check(_B.lib().bsgp_extract_tiles(_B._ptr(img), H, W, _B._ptr(bd), len(b), th, tw,
                                         _B._ptr(out), _B.current_stream()))
    out._keep = (img, bd)
    return out


def coadd_tiles(tiles, boxes, shape):
    """Mean mosaic [H, W] and footprint [H, W] (tiles covering each pixel)."""
    _B.require_gpu()
    torch = _B.torch
    t = tiles if torch.is_tensor(tiles) else _B.to_dev(np.asarray(tiles, dtype=np.float64))
    t = t.to(dtype=torch.float64).contiguous()
    n, th, tw = t.shape
    b = np.asarray(boxes, dtype=np.int32).reshape(-1, 4)
    if len(b) != n:
        raise ValueError("one box per tile")
    bd = torch.from_numpy(np.ascontiguousarray(b)).to("cuda")
    H, W = shape
    mean = torch.empty((H, W), dtype=torch.float64, device="cuda")
    foot = torch.empty((H, W), dtype=torch.float64, device="cuda")
    _B.check(_B.lib().bsgp_coadd_tiles(_B._ptr(t), n, th, tw, _B._ptr(bd), H, W, _B._ptr(mean),
                                       _B._ptr(foot), _B.current_stream()))
    mean._keep = (t, bd)
    return mean, foot


def sgp_subdivisions(image, psf, bkg, subdiv_shape=(256, 256), overlap=32, betaParams=None,
                     device_out=False, **sgp_kwargs):
    """Field -> overlapping subdivisions -> one batched beta-SGP solve -> mean
    mosaic.  ``bkg``: scalar, or a field-sized map (cut like the image, as the
    application cuts its background map).  ``psf``: one stamp for every tile,
    [n_tiles, kh, kw] stamps, or a DIAPL model (psf_calculate.PSF), which is
    evaluated on the device at every tile centre (field pixel coordinates,
    (x, y) = ((x0 + x1 - 1) / 2, (y0 + y1 - 1) / 2)) so each tile is solved
    with its own PSF.  Returns (mosaic, footprint, solve outputs); numpy
    unless device_out."""
    import sgp
    torch = _B.torch
    img = _field(image)
    H, W = img.shape
    boxes = subdivision_boxes((H, W), subdiv_shape, overlap)
    tiles = extract_tiles(img, boxes, subdiv_shape)
    b = np.asarray(bkg) if not torch.is_tensor(bkg) else bkg
    if (torch.is_tensor(b) and b.dim() == 2) or (not torch.is_tensor(b) and b.ndim == 2):
        bk = extract_tiles(b, boxes, subdiv_shape)
    else:
        bk = torch.full((len(boxes),), float(b), dtype=torch.float64, device="cuda")
    if hasattr(psf, "stamps"):  # spatially varying DIAPL model: a stamp per tile centre
        psf = psf.stamps(tile_centres(boxes), normalize=True, device_out=True)
    out = sgp.sgp_betaDiv_batch(tiles, psf, bk, betaParams=betaParams, device_out=True,
                                **sgp_kwargs)
    mosaic, foot = coadd_tiles(out["x"], boxes, (H, W))
    if device_out:
        return mosaic, foot, out
    torch.cuda.current_stream().synchronize()
    _B.check_status(out["counters"])
    return mosaic.cpu().numpy(), foot.cpu().numpy(), \
        {k: (v.cpu().numpy() if v is not None else None) for k, v in out.items()}
