"""Pure-Python model of the row-unit SpMM schedule (test infrastructure).

Mirrors, step by step, the host unit planning (spmm.hip host_plan, row part:
light rows, heavy rows cut at XCD column-class boundaries and into segments,
the class-by-workgroup layout with empty padding units) and the row kernel's
control flow (light units per lane group, heavy segments shared by lane
groups, partial slots and the last-arriver combine in segment order; rows of
more than K_MAX_SEG segments in groups whose last arrivers publish the group
sums into the row's top entry, summed by spmm_heavy_top_kernel after the
launch), so the control logic can be checked on CPU against a dense product."""
import numpy as np

K_MAX_SEG = 64
K_MAX_SEG_ROW = K_MAX_SEG * K_MAX_SEG
NX = 8


def _cls(i, n):
    return i * NX // n if n > 0 else 0


def geometry(groups):
    lpr = 64 // groups
    block = 256 if lpr >= 8 else 64
    wpb, sg = block // 64, block // lpr
    wg_heavy = lpr == 64 or (lpr >= 8 and wpb > 1)   # a heavy segment spans the workgroup
    hpb = 1 if wg_heavy else wpb
    seg_groups = wpb if lpr == 64 else groups * (wpb if wg_heavy else 1)
    lpb = 2 * sg if lpr == 64 else sg  # light units per workgroup (two per wavefront at 64 lanes)
    return hpb, lpb, seg_groups, lpr


def host_plan(rowptr, colind, K, ipc, groups):
    """-> (units [(row, b, e, w)], heavy [(row, first slot, slots, w)], nh, nslots); heavy w: -1 one
    level, -2 a top entry (slots = its groups' sums), >= 0 a group (w = the top's slot for its sum)."""
    hpb, lpb, seg_groups, lpr = geometry(groups)
    seg = ipc * seg_groups
    light_max = min(2 * ipc, 32) if lpr == 64 else ipc
    M = len(rowptr) - 1
    hq, lq, heavy = [[] for _ in range(NX)], [[] for _ in range(NX)], []
    nslots = 0
    rr_class = 0
    for r in range(M):
        b, e = int(rowptr[r]), int(rowptr[r + 1])
        deg = e - b
        if deg <= light_max:
            lq[_cls(r, M)].append((r, b, e, -1))
            continue
        runs = []
        if deg * 2 >= seg * NX:
            for k in range(b, e):
                c = _cls(int(colind[k]), K)
                if not runs or runs[-1][1] != c:
                    runs.append([k, c])
        if not runs or len(runs) > NX:
            runs = [[b, rr_class % NX]]
            rr_class += 1
        bounds = [x[0] for x in runs] + [e]
        sr = seg
        while True:
            nseg = sum((bounds[i + 1] - bounds[i] + sr - 1) // sr for i in range(len(runs)))
            if nseg <= K_MAX_SEG_ROW:
                break
            sr *= 2
        if nseg == 1:
            hq[runs[0][1]].append((r, b, e, -1))
            continue
        ng = 1 if nseg <= K_MAX_SEG else (nseg + K_MAX_SEG - 1) // K_MAX_SEG
        top_slot = -1
        if ng > 1:
            heavy.append((r, nslots, ng, -2))
            top_slot = nslots
            nslots += ng
        seg_w = [0] * nseg
        for g in range(ng):
            s0, s1 = g * nseg // ng, (g + 1) * nseg // ng
            hid = len(heavy)
            heavy.append((r, nslots, s1 - s0, top_slot + g if ng > 1 else -1))
            for sgi in range(s0, s1):
                seg_w[sgi] = hid * 64 + sgi - s0
            nslots += s1 - s0
        sgi = 0
        for i, (pb, c) in enumerate(runs):
            ln = bounds[i + 1] - pb
            npc = (ln + sr - 1) // sr
            for s in range(npc):
                hq[c].append((r, pb + ln * s // npc, pb + ln * (s + 1) // npc, seg_w[sgi]))
                sgi += 1

    def layout(qs, per):
        out = []
        rounds = max((len(q) + per - 1) // per for q in qs)
        for k in range(rounds):
            for c in range(NX):
                for j in range(per):
                    i = k * per + j
                    out.append(qs[c][i] if i < len(qs[c]) else (-1, 0, 0, -1))
        return out

    units = layout(hq, hpb)
    nh = len(units)
    units += layout(lq, lpb)
    return units, heavy, nh, nslots


def spmm(rowptr, colind, val, B, ipc, groups):
    """C = A @ B computed the way the row kernel schedules it (float64), with
    the per-workgroup XCD class of every unit checked."""
    M, K = len(rowptr) - 1, B.shape[0]
    hpb, lpb, seg_groups, _ = geometry(groups)
    units, heavy, nh, nslots = host_plan(rowptr, colind, K, ipc, groups)
    C = np.full((M, B.shape[1]), np.nan)
    part = np.zeros((nslots, B.shape[1]))
    arrivals = [0] * len(heavy)
    written = np.zeros(M, np.int64)

    def gather(b, e, q, stride):
        acc = np.zeros(B.shape[1])
        for k in range(b + q, e, stride):
            acc += val[k] * B[colind[k]]
        return acc

    # heavy region (workgroup u // hpb); arrivals in an arbitrary (reversed) order
    for u in reversed(range(nh)):
        r, b, e, w = units[u]
        if r < 0:
            continue
        acc = sum(gather(b, e, q, seg_groups) for q in range(seg_groups))
        if w < 0:
            C[r] = acc
            written[r] += 1
            continue
        hid, slot = w >> 6, w & 63
        hr, first, nsl, up = heavy[hid]
        assert nsl <= K_MAX_SEG, "no combine reads more than K_MAX_SEG partials"
        part[first + slot] = acc
        arrivals[hid] += 1
        if arrivals[hid] == nsl:        # last arriver: slots in segment order
            gsum = sum(part[first + s] for s in range(nsl))
            if up >= 0:                 # a group of a long row: into the top entry's slot
                part[up] = gsum
            else:
                C[hr] = gsum
                written[hr] += 1
    for hr, first, nsl, up in heavy:    # after the launch: spmm_heavy_top_kernel
        if up == -2:
            C[hr] = sum(part[first + s] for s in range(nsl))
            written[hr] += 1
    for u in range(nh, len(units)):
        r, b, e, _ = units[u]
        if r < 0:
            continue
        assert ((nh // hpb + (u - nh) // lpb) % NX) == _cls(r, M), "light unit in its XCD class"
        C[r] = gather(b, e, 0, 1)
        written[r] += 1
    assert np.all(written == 1), "every row is stored exactly once"
    return C
