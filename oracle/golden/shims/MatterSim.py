"""Offline stand-in for the MatterSim pybind module (test infrastructure, container only).

Emulates only the discretized 12x3 view state machine of MatterSim.cpp:339-367 / 470-508 that
r2r_src/utils.py (ViewHelper, get_point_angle_feature) drives at import time. No rendering, no
navigation graph: navigableLocations holds only the current location.
"""
import math

_HINC = 2 * math.pi / 12
_EINC = math.pi / 6


class _Loc:
    def __init__(self, vid):
        self.viewpointId = vid
        self.rel_heading = 0.0
        self.rel_elevation = 0.0
        self.rel_distance = 0.0


class _State:
    pass


class Simulator:
    def __init__(self):
        self.heading = 0.0
        self.elevation = 0.0
        self.viewIndex = 0
        self.vp = ""
        self.scan = ""

    def setRenderingEnabled(self, v): pass
    def setCameraResolution(self, w, h): pass
    def setCameraVFOV(self, v): pass
    def setDiscretizedViewingAngles(self, v): pass
    def setBatchSize(self, v): pass
    def setNavGraphPath(self, v): pass
    def init(self): pass
    def initialize(self): pass

    def _set(self, heading, elevation):
        h = math.fmod(heading, 2 * math.pi)
        while h < 0:
            h += 2 * math.pi
        step = int(math.floor(h / _HINC + 0.5))
        if step == 12:
            step = 0
        self.heading = step * _HINC
        if elevation < -_EINC / 2:
            self.elevation, self.viewIndex = -_EINC, step
        elif elevation > _EINC / 2:
            self.elevation, self.viewIndex = _EINC, step + 24
        else:
            self.elevation, self.viewIndex = 0.0, step + 12

    def newEpisode(self, scan, vp, heading, elevation):
        self.scan, self.vp = scan, vp
        self._set(heading, elevation)

    def makeAction(self, index, heading, elevation):
        h = _HINC if heading > 0 else (-_HINC if heading < 0 else 0.0)
        e = _EINC if elevation > 0 else (-_EINC if elevation < 0 else 0.0)
        self._set(self.heading + h, self.elevation + e)

    def getState(self):
        s = _State()
        s.scanId, s.location = self.scan, _Loc(self.vp)
        s.heading, s.elevation, s.viewIndex = self.heading, self.elevation, self.viewIndex
        s.navigableLocations = [_Loc(self.vp)]
        return s
