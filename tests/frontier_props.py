"""Topological properties of cv::findContours(RETR_EXTERNAL, CHAIN_APPROX_NONE)
(src/safe_bayesian_optimization_node.cpp:461-462) checked WITHOUT any border
follower: connected components and background regions come from
scipy.ndimage.label, so these checks are independent of the Suzuki-Abe
transcriptions in csrc/frontier.cpp and oracle/sbo_oracle.c.

Semantics restated (Suzuki & Abe 1985, the algorithm OpenCV implements; the
image is zero-padded by one pixel, as OpenCV >= 3.2 does):
  * foreground is 8-connected, background 4-connected;
  * RETR_EXTERNAL keeps the outer border of every foreground component that
    is not inside a hole of another component -- i.e. of every component
    4-adjacent to the background region that contains the padding;
  * the outer border of such a component C is the set of pixels of C with a
    4-neighbour in that outer background region (a border point between C
    and the region);
  * CHAIN_APPROX_NONE emits every traversed border pixel: a contour is a
    closed 8-connected walk (consecutive points 8-adjacent, the last adjacent
    to the first), it starts at C's first pixel in raster order (where the
    raster scan finds the border), and a pixel passed twice -- a 1-px wide
    line -- is emitted twice.
Test helper, not product code."""
import numpy as np
from scipy import ndimage

EIGHT = np.ones((3, 3), bool)
FOUR = ndimage.generate_binary_structure(2, 1)


def expected_borders(img):
    """For a (h, w) mask: (labels of the 8-connected foreground components,
    {label: (first raster pixel (x, y), set of outer-border pixels (x, y))}
    for the components RETR_EXTERNAL reports)."""
    fg = np.asarray(img) != 0
    h, w = fg.shape
    lab, n = ndimage.label(fg, structure=EIGHT)
    bgp = np.pad(~fg, 1, constant_values=True)
    blab, _ = ndimage.label(bgp, structure=FOUR)
    outer = (blab == blab[0, 0])[1:-1, 1:-1] if h and w else np.zeros_like(fg)
    outer_p = np.pad(outer, 1, constant_values=True)
    # pixels of fg with a 4-neighbour in the outer background (padding included)
    nb = (outer_p[:-2, 1:-1] | outer_p[2:, 1:-1] | outer_p[1:-1, :-2] | outer_p[1:-1, 2:])
    border = fg & nb
    res = {}
    ys, xs = np.nonzero(border)
    for y, x in zip(ys.tolist(), xs.tolist()):
        res.setdefault(int(lab[y, x]), set()).add((x, y))
    out = {}
    for lb, pix in res.items():
        cy, cx = np.nonzero(lab == lb)
        first = int(np.argmin(cy * w + cx))
        out[lb] = ((int(cx[first]), int(cy[first])), pix)
    return lab, out


def check_contours(img, contours):
    """Assert the properties above for a list of (k, 2) (x, y) contours."""
    lab, exp = expected_borders(img)
    assert len(contours) == len(exp), (len(contours), len(exp))
    seen = set()
    for c in contours:
        c = np.asarray(c)
        assert c.ndim == 2 and c.shape[1] == 2 and len(c) > 0
        labels = {int(lab[y, x]) for x, y in c.tolist()}
        assert len(labels) == 1 and 0 not in labels, labels     # one component, foreground only
        lb = labels.pop()
        assert lb in exp and lb not in seen, lb                # a reported component, once
        seen.add(lb)
        first, pix = exp[lb]
        assert tuple(c[0].tolist()) == first                   # starts where the raster scan meets C
        assert set(map(tuple, c.tolist())) == pix              # exactly C's outer border
        if len(c) > 1:
            d = np.abs(np.diff(np.vstack([c, c[:1]]), axis=0)).max(axis=1)
            assert np.all(d == 1), d                           # closed 8-connected walk
    return lab, exp


def check_flat_frontier(img, pixels):
    """The frontier as the node sees it (FindSafetyContourIndices flattens the
    contours): the same pixel set, and at most
    #contours - 1 breaks in 8-adjacency between consecutive pixels."""
    lab, exp = expected_borders(img)
    pixels = np.asarray(pixels).reshape(-1, 2)
    want = set().union(*[p for _, p in exp.values()]) if exp else set()
    assert set(map(tuple, pixels.tolist())) == want
    if len(pixels) > 1:
        d = np.abs(np.diff(pixels, axis=0)).max(axis=1)
        assert np.count_nonzero(d > 1) <= len(exp) - 1
    return exp
