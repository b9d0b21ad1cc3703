"""Inert stand-in for CCBlade (absent from the image).  Golden cases use wind_speed=0,
so rotor aerodynamics are never evaluated (reference raft/raft_fowt.py:801)."""


class CCAirfoil:
    def __init__(self, *a, **kw):
        pass


class CCBlade:
    def __init__(self, *a, **kw):
        self.args = a
        self.kw = kw
