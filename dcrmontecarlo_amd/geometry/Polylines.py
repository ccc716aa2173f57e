"""Abstract polyline boundary (reference: geometry/Polylines.py:8-63).

Same interface: ``PolyLines(points)`` holds its ``[N,2]`` vertex array by
reference, supports ``len`` and indexing, and declares the five queries the
Walk-on-Stars step needs. Subclasses implement them.
"""
from __future__ import annotations


class PolyLines:
    """A polyline in 2-D given by consecutive vertices ``points[N,2]``."""

    def __init__(self, points):
        self.points = points                      # held by reference (Polylines.py:21)

    def __len__(self):
        return self.points.shape[0]

    def __getitem__(self, idx):
        return self.points[idx]

    def distance(self, point):
        raise NotImplementedError("Subclasses should implement this method.")

    def isSilhouette(self, point):
        raise NotImplementedError("Subclasses should implement this method.")

    def silhouetteDistance(self, point):
        raise NotImplementedError("Subclasses should implement this method.")

    def rayIntersection(self, point, direction):
        raise NotImplementedError("Subclasses should implement this method.")

    def intersectPolylines(self, point, direction, r):
        raise NotImplementedError("Subclasses should implement this method.")
