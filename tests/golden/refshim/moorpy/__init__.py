"""Inert stand-in for MoorPy, used ONLY by tests/golden/make_golden.py to import the
read-only reference (/root/reference/raft) inside the build container.

MoorPy is not installed in this image.  Nothing here is on the hot
path: mooring stiffness enters the response solve as an input matrix (C_moor), which the
golden generator sets explicitly from a fixed fixture after setPosition().  Mean mooring
forces are zero.  This module is never imported by the product or by GPU tests.
"""
import numpy as np

__all__ = ["System", "Body", "Point"]


class Point:
    def __init__(self, number, ptype, r):
        self.number = number
        self.type = ptype
        self.r = np.array(r, dtype=float)


class Body:
    def __init__(self, btype=-1, r6=None):
        self.type = btype
        self.r6 = np.zeros(6) if r6 is None else np.array(r6, dtype=float)
        self.attachedP = []

    def attachPoint(self, number, r):
        self.attachedP.append(number)

    def setPosition(self, r6):
        self.r6 = np.array(r6, dtype=float)

    def getForces(self, lines_only=False, **kw):
        return np.zeros(6)

    def getStiffness(self, *a, **kw):
        return np.zeros((6, 6))


class System:
    def __init__(self, depth=0.0, **kw):
        self.depth = depth
        self.bodyList = []
        self.pointList = []
        self.lineList = []

    def parseYAML(self, d):
        # keep the line count so per-line outputs have the right shape; no physics
        self.lineList = list(d.get("lines", [])) if isinstance(d, dict) else []

    def addBody(self, btype, r6, **kw):
        self.bodyList.append(Body(btype, r6))

    def transform(self, *a, **kw):
        pass

    def initialize(self, *a, **kw):
        pass

    def solveEquilibrium(self, *a, **kw):
        return True

    def getCoupledStiffnessA(self, *a, **kw):
        n = 6 * max(1, len(self.bodyList))
        return np.zeros((n, n))

    def getCoupledStiffness(self, *a, tensions=False, **kw):
        n = 6 * max(1, len(self.bodyList))
        if tensions:
            return np.zeros((n, n)), np.zeros((2 * len(self.lineList), n))
        return np.zeros((n, n))

    def getTensions(self):
        return np.zeros(2 * len(self.lineList))

    def getForces(self, *a, **kw):
        return np.zeros(6 * max(1, len(self.bodyList)))

    def load(self, *a, **kw):
        pass
