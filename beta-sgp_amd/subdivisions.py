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


def _check_bkg_dtype(gn_f32, bkg):
    """A float32 field keeps the reference's float32 arithmetic, where numpy
    also computes the background's share (bkg scaling, sgp.py:648-666) in the
    background's own dtype: tiles cut from a float32 / integer background would
    reach the solve already widened to float64 and silently lose that parity,
    so they raise here as sgp_betaDiv_batch raises for such backgrounds."""
    torch = _B.torch
    if not gn_f32:
        return
    dt = bkg.dtype if torch.is_tensor(bkg) else np.asarray(bkg).dtype
    f64 = dt == torch.float64 if torch.is_tensor(bkg) else (dt.kind == "f" and dt.itemsize == 8)
    if not f64:
        raise ValueError("float32 images in a batch need float64 backgrounds (numpy computes the "
                         "background's part in float32 from a float32 background; solve such "
                         "images one at a time with sgp_betaDiv / sgp)")


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
    # a float32 field (the application's FITS data) keeps the reference's
    # float32 arithmetic per tile (sgp.py:648-666; include/bsgp.h gn_f32)
    f32 = (image.dtype == torch.float32) if torch.is_tensor(image) else \
        (np.asarray(image).dtype.kind == "f" and np.asarray(image).dtype.itemsize == 4)
    sgp_kwargs.setdefault("gn_f32", bool(f32))
    _check_bkg_dtype(sgp_kwargs["gn_f32"], bkg)
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


def sgp_subdivisions_multistart(image, psf, bkg, betas=None, score=None, subdiv_shape=(256, 256),
                                overlap=32, **sgp_kwargs):
    """The application's beta search for every subdivision of a field at once
    (application_sgp_subdivisions.py:69-107 per tile): the (tile x candidate)
    product -- n tiles x K initial betas (default: the application's five
    seeds) -- is ONE batched solve, image t*K + k being tile t with beta k;
    each tile keeps the candidate its score ranks best with the application's
    strict running minimum (sgp.argmin_strict), and the mosaic is co-added
    from those.  The application's final re-solve with the best beta repeats
    that candidate's run exactly (the reference is deterministic), so it is
    not run again.

    ``score(x, tile)`` (host arrays of one candidate and its observed tile)
    stands in for the application's photometric score (photutils, absent
    here); without one the final discrepancy ranks the candidates.  ``psf``,
    ``bkg`` and the keyword arguments as in :func:`sgp_subdivisions`.
    Returns (mosaic, footprint, info): info holds the boxes, "betas",
    "scores" [n, K], "best" [n] (candidate index per tile), "best_beta" [n],
    and the solve outputs of the chosen candidates ("x", "iters", "discr",
    "beta_final")."""
    import sgp
    torch = _B.torch
    betas = list(sgp.app_beta_candidates() if betas is None else betas)
    K = len(betas)
    f32 = (image.dtype == torch.float32) if torch.is_tensor(image) else \
        (np.asarray(image).dtype.kind == "f" and np.asarray(image).dtype.itemsize == 4)
    sgp_kwargs.setdefault("gn_f32", bool(f32))
    _check_bkg_dtype(sgp_kwargs["gn_f32"], bkg)
    img = _field(image)
    H, W = img.shape
    boxes = subdivision_boxes((H, W), subdiv_shape, overlap)
    n = len(boxes)
    tiles = extract_tiles(img, boxes, subdiv_shape)
    b = np.asarray(bkg) if not torch.is_tensor(bkg) else bkg
    if (torch.is_tensor(b) and b.dim() == 2) or (not torch.is_tensor(b) and b.ndim == 2):
        bk = extract_tiles(b, boxes, subdiv_shape).repeat_interleave(K, dim=0)
    else:
        bk = torch.full((n * K,), float(b), dtype=torch.float64, device="cuda")
    if hasattr(psf, "stamps"):
        psf = psf.stamps(tile_centres(boxes), normalize=True, device_out=True)
    if (psf.dim() if torch.is_tensor(psf) else np.ndim(psf)) == 3:
        pt = psf if torch.is_tensor(psf) else _B.to_dev(np.asarray(psf, dtype=np.float64))
        psf = pt.repeat_interleave(K, dim=0)
    gns = tiles.repeat_interleave(K, dim=0)
    out = sgp.sgp_betaDiv_batch(gns, psf, bk, betaParams=np.tile(np.asarray(betas, float), n),
                                **sgp_kwargs)
    t_host = tiles.cpu().numpy()
    scores = np.empty((n, K))
    for t in range(n):
        for k in range(K):
            i = t * K + k
            it = int(out["iters"][i])
            scores[t, k] = (float(score(out["x"][i], t_host[t])) if score is not None
                            else float(out["discr"][i, it]))
    best = []
    for t in range(n):
        j = sgp.argmin_strict(scores[t])
        if j is None:
            raise ValueError(f"tile {t}: no candidate scores below +inf ({scores[t]})")
        best.append(j)
    best = np.asarray(best)
    pick = np.arange(n) * K + best
    xs = out["x"][pick]
    mosaic, foot = coadd_tiles(xs, boxes, (H, W))
    info = {"boxes": boxes, "betas": betas, "scores": scores, "best": best,
            "best_beta": np.asarray(betas)[best], "x": xs, "iters": out["iters"][pick],
            "discr": out["discr"][pick], "beta_final": out["beta_final"][pick]}
    torch.cuda.current_stream().synchronize()
    return mosaic.cpu().numpy(), foot.cpu().numpy(), info
