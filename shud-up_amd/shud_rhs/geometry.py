"""Derived element / river geometry, restating the reference's setup code (vectorised numpy).

Same fp64 operation order as the reference so the derived SoA equals what Model_Data::initialize()
computes:  _Element::applyGeometry (src/classes/Element.cpp:62-217), applyNabor (:238-270),
InitElement (:218-237), Model_Data::rmSinks (src/ModelData/Model_Data.cpp:238-266),
_Node::Init (src/classes/Node.cpp:13-20), _River::updateFrDownstream (src/classes/River.cpp:74-84).
"""
import heapq

import numpy as np


def eudist(x1, y1, x2, y2):
    """functions.hpp Eudist: sqrt(dx*dx + dy*dy) with dx = x2 - x1."""
    dx = x2 - x1
    dy = y2 - y1
    return np.sqrt(dx * dx + dy * dy)


def point_perp_on_line(x, y, x1, y1, x2, y2):
    """functions.cpp:259-288 PointPerpdicularOnLine (closest point of segment (x1,y1)-(x2,y2))."""
    A = x - x1
    B = y - y1
    Cc = x2 - x1
    D = y2 - y1
    dot = A * Cc + B * D
    len_sq = Cc * Cc + D * D
    with np.errstate(divide="ignore", invalid="ignore"):
        param = np.where(len_sq != 0, dot / np.where(len_sq != 0, len_sq, 1.0), -1.0)
    xx = np.where(param < 0.0, x1, np.where(param > 1.0, x2, x1 + param * Cc))
    yy = np.where(param < 0.0, y1, np.where(param > 1.0, y2, y1 + param * D))
    return xx, yy


def node_zmin(zmax, aqd, c_aqd=0.0):
    """Node.cpp:13-20: zmin = zmax - (AqD + cAqD)."""
    return zmax - (aqd + c_aqd)


def element_geometry(nx, ny, nzmax, nzmin, tri):
    """Element.cpp:62-121 for all elements.  tri: [NE,3] 0-based node indices (anticlockwise)."""
    i1, i2, i3 = tri[:, 0], tri[:, 1], tri[:, 2]
    x1, x2, x3 = nx[i1], nx[i2], nx[i3]
    y1, y2, y3 = ny[i1], ny[i2], ny[i3]
    area = 0.5 * ((x2 - x1) * (y3 - y1) - (y2 - y1) * (x3 - x1))
    z_surf = (nzmax[i1] + nzmax[i2] + nzmax[i3]) / 3.0
    z_bottom = (nzmin[i1] + nzmin[i2] + nzmin[i3]) / 3.0
    x = (x1 + x2 + x3) / 3.0
    y = (y1 + y2 + y3) / 3.0
    edge = np.stack([eudist(x2, y2, x3, y3), eudist(x3, y3, x1, y1), eudist(x1, y1, x2, y2)])
    p1 = point_perp_on_line(x, y, x2, y2, x3, y3)
    p2 = point_perp_on_line(x, y, x3, y3, x1, y1)
    p3 = point_perp_on_line(x, y, x1, y1, x2, y2)
    d2e = np.stack([eudist(p1[0], p1[1], x, y), eudist(p2[0], p2[1], x, y), eudist(p3[0], p3[1], x, y)])
    return dict(area=area, z_surf=z_surf, z_bottom=z_bottom, x=x, y=y, edge=edge, dist2edge=d2e)


def apply_nabor(nabr, x, y, rough, dist2edge):
    """Element.cpp:238-270.  nabr: [3,NE] 0-based (-1 boundary).  Returns dist2nabor, avg_rough [3,NE]."""
    d2n = np.zeros(nabr.shape)
    avg = np.zeros(nabr.shape)
    for j in range(3):
        nb = nabr[j]
        has = nb >= 0
        nbs = np.where(has, nb, 0)
        d2n[j] = np.where(has, eudist(x, y, x[nbs], y[nbs]), 0.0)
        avg[j] = np.where(has, 0.5 * (rough + rough[nbs]), rough)
    return d2n, avg


def rm_sinks(z_surf, z_bottom, aq, nabr, riv_id):
    """Model_Data.cpp:238-266 (in-place, sequential in element order like the reference loop).

    Raising element i changes the neighbour minimum of later elements, so after the vectorised first
    pass the candidates are processed in ascending order with a heap, re-testing neighbours > i."""
    NE = z_surf.size
    z_surf = z_surf.copy()
    z_bottom = z_bottom.copy()
    big = 1.0e200

    def zmin_nb(i):
        m = big
        for j in range(3):
            nb = nabr[j, i]
            if nb >= 0:
                v = z_surf[nb]
                m = v if m > v else m          # min(a,b) = a > b ? b : a
        return m

    zn = np.full(NE, big)
    for j in range(3):
        nb = nabr[j]
        v = np.where(nb >= 0, z_surf[np.where(nb >= 0, nb, 0)], big)
        zn = np.where(zn > v, v, zn)
    cand = list(np.nonzero((zn > z_surf) & (riv_id <= 0))[0])
    heapq.heapify(cand)
    done = set()
    raised = []
    while cand:
        i = int(heapq.heappop(cand))
        if i in done:
            continue
        done.add(i)
        m = zmin_nb(i)
        if m > z_surf[i] and riv_id[i] <= 0:
            z_surf[i] = m
            z_bottom[i] = m - aq[i]
            raised.append(i)
            for j in range(3):
                nb = nabr[j, i]
                if nb > i and nb not in done:
                    heapq.heappush(cand, int(nb))
    return z_surf, z_bottom, raised


def river_downstream(down, length, riv_rough):
    """River.cpp:74-84 updateFrDownstream: avgRough and Dist2DownStream (down 0-based, <0 outlet)."""
    has = down >= 0
    d = np.where(has, down, 0)
    avg = np.where(has, 0.5 * (riv_rough + riv_rough[d]), riv_rough)
    dist = np.where(has, 0.5 * (length + length[d]), length)
    return avg, dist
