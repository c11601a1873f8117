"""Pure-Python model of the row-unit SpMM schedule (test infrastructure).

Mirrors, step by step, the host unit planning (spmm.hip host_plan, row part)
and the row kernel's control flow (light units per lane group, heavy segments
per wavefront with lane groups on interleaved nonzeros, partial slots and the
last-arriver combine in segment order), so the control logic can be checked on
CPU against a dense product."""
import numpy as np

K_MAX_SEG = 64


def host_plan(rowptr, ipc, groups, tile_rows=()):
    """-> (units [(row, b, e, hid)], heavy [(row, first unit, nseg)], nh)."""
    seg = ipc * groups
    tile = set(tile_rows)
    heavy_units, light, heavy = [], [], []
    for r in range(len(rowptr) - 1):
        if r in tile:
            continue
        b, deg = int(rowptr[r]), int(rowptr[r + 1] - rowptr[r])
        if deg <= ipc:
            light.append((r, b, b + deg, -1))
            continue
        nseg = min((deg + seg - 1) // seg, K_MAX_SEG)
        hid = len(heavy) if nseg > 1 else -1
        if nseg > 1:
            heavy.append((r, len(heavy_units), nseg))
        for s in range(nseg):
            heavy_units.append((r, b + deg * s // nseg, b + deg * (s + 1) // nseg, hid))
    return heavy_units + light, heavy, len(heavy_units)


def spmm(rowptr, colind, val, B, ipc, groups):
    """C = A @ B computed the way the row kernel schedules it (float64)."""
    M = len(rowptr) - 1
    units, heavy, nh = host_plan(rowptr, ipc, groups)
    C = np.full((M, B.shape[1]), np.nan)
    part = np.zeros((nh, B.shape[1]))
    arrivals = [0] * len(heavy)
    written = np.zeros(M, np.int64)

    def gather(b, e, q, stride):
        acc = np.zeros(B.shape[1])
        for k in range(b + q, e, stride):
            acc += val[k] * B[colind[k]]
        return acc

    # heavy segments first (grid order), each wavefront's lane groups interleave
    # nonzeros; arrivals in an arbitrary (here reversed) order
    for u in reversed(range(nh)):
        r, b, e, hid = units[u]
        acc = sum(gather(b, e, q, groups) for q in range(groups))
        if hid < 0:
            C[r] = acc
            written[r] += 1
            continue
        part[u] = acc
        arrivals[hid] += 1
        hr, first, nseg = heavy[hid]
        if arrivals[hid] == nseg:       # last arriver: slots in segment order
            C[hr] = sum(part[first + s] for s in range(nseg))
            written[hr] += 1
    for u in range(nh, len(units)):
        r, b, e, _ = units[u]
        C[r] = gather(b, e, 0, 1)
        written[r] += 1
    assert np.all(written == 1), "every row is stored exactly once"
    return C
