"""Inert stand-ins for the three moorpy.helpers names the reference imports.
transformPosition follows MoorPy's published definition: r6[:3] + R(r6[3:]) @ r."""
import numpy as np


def _rot(x3, x2, x1):
    s1, c1 = np.sin(x1), np.cos(x1)
    s2, c2 = np.sin(x2), np.cos(x2)
    s3, c3 = np.sin(x3), np.cos(x3)
    return np.array([[c1 * c2, c1 * s2 * s3 - c3 * s1, s1 * s3 + c1 * c3 * s2],
                     [c2 * s1, c1 * c3 + s1 * s2 * s3, c3 * s1 * s2 - c1 * s3],
                     [-s2, c2 * s3, c2 * c3]])


def transformPosition(rRelBody, r6):
    return np.array(r6[:3], dtype=float) + _rot(*r6[3:]) @ np.array(rRelBody, dtype=float)


def dsolve2(*a, **kw):
    raise RuntimeError("dsolve2 (MoorPy statics) is not available in this container")


def set_axes_equal(*a, **kw):
    pass


def dsolvePlot(*a, **kw):
    pass
