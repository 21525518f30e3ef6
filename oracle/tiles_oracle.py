"""TEST INFRASTRUCTURE — numpy restatement of the data paths either side of the
solver, the checker for beta-sgp_amd/subdivisions.py and
beta-sgp_amd/fits_io.py.  Only tests/, __graft_entry__.smoke() and bench.py's
CPU leg use it; the product never imports it.

Pinned by tests/golden/make_golden_io.py: the reference's own
calculate_slice_bboxes (restoration/utils.py:332-372) on 8 cases and astropy
4.3.1 Cutout2D / astropy.io.fits on the reference's data files.
"""
import numpy as np


def calculate_slice_bboxes(image_height, image_width, slice_height=512, slice_width=512,
                           overlap_height_ratio=0.2, overlap_width_ratio=0.2):
    """utils.py:332-372: xyxy boxes of overlapping slices, row-major; the last
    slice of a row/column is shifted back inside the image.  Overlaps are
    int(ratio * size) (utils.py:357-358), so create_subdivisions' ratio
    overlap/size can lose a pixel to rounding."""
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
                xmin = max(0, xmax - slice_width)
                ymin = max(0, ymax - slice_height)
                boxes.append([xmin, ymin, xmax, ymax])
            else:
                boxes.append([x_min, y_min, x_max, y_max])
            x_min = x_max - x_overlap
        y_min = y_max - y_overlap
    return boxes


def extract_tiles(image, boxes):
    """Cutout2D(image, centre, size) of create_subdivisions (utils.py:375-386)
    for boxes of exactly the tile size: plain slices."""
    return np.stack([image[y0:y1, x0:x1] for x0, y0, x1, y1 in boxes])


def coadd_mean(tiles, boxes, shape):
    """Mean co-add in tile order (the same-WCS case of reproject_and_coadd,
    utils.py:389-395, combine_function='mean', no background matching)."""
    s = np.zeros(shape)
    c = np.zeros(shape)
    for t, (x0, y0, x1, y1) in zip(tiles, boxes):
        s[y0:y1, x0:x1] += t
        c[y0:y1, x0:x1] += 1.0
    out = np.zeros(shape)
    np.divide(s, c, out=out, where=c > 0)
    return out, c
