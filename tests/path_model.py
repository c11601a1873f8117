"""Pure-Python model of the path-format SpMM schedule (test infrastructure).

Mirrors, step by step, the host window packing (spmm.hip host_plan) and the
kernel's per-group walk, in-window combine and cross-window fix-up, so the
control logic can be checked on CPU against a dense product."""
import numpy as np

MARKER, PAD = -1, -2


def host_plan(rowptr, W):
    M = len(rowptr) - 1
    heavy = W // 2
    start = np.zeros(M, np.int64)
    pos = 0
    for r in range(M):
        ln = rowptr[r + 1] - rowptr[r] + 1
        off = pos % W
        if ln <= heavy and off + ln > W:
            pos += W - off
        start[r] = pos
        pos += ln
    nwin = (pos + W - 1) // W
    head = [-1] * nwin
    tail = [-1] * nwin
    cross = []
    for r in range(M):
        a = start[r]
        e = a + (rowptr[r + 1] - rowptr[r])
        wa, wb = a // W, e // W
        if wa < wb:
            cross.append((r, wa, wb))
    for r, wa, wb in cross:
        for x in range(wa, wb):
            tail[x] = 1
        head[wb] = 1
    slot = 0
    for x in range(nwin):
        if head[x] >= 0:
            head[x] = slot
            slot += 1
        if tail[x] >= 0:
            tail[x] = slot
            slot += 1
    fix = [(r, tail[wa], head[wb]) for r, wa, wb in cross]
    return start, nwin, head, tail, fix, slot


def items_of(rowptr, colind, val, start, nwin, W):
    items = [(PAD, 0.0)] * (nwin * W)
    for r in range(len(rowptr) - 1):
        b, e = rowptr[r], rowptr[r + 1]
        s = start[r]
        for k in range(b, e):
            items[s + k - b] = (int(colind[k]), float(val[k]))
        items[s + e - b] = (MARKER, r)
    return items


def spmm(rowptr, colind, val, B, G, ipc):
    W = G * ipc
    M = len(rowptr) - 1
    F = B.shape[1]
    start, nwin, head, tail, fix, nslots = host_plan(rowptr, W)
    items = items_of(rowptr, colind, val, start, nwin, W)
    C = np.full((M, F), np.nan)
    part = np.full((max(nslots, 1), F), np.nan)
    for w in range(nwin):
        base = w * W
        s_item = [items[base - 1] if w > 0 else (MARKER, -1)] + items[base:base + W]
        meta = []
        H = [None] * G
        T = [None] * G
        for g in range(G):
            i0 = 1 + g * ipc
            head_partial = s_item[i0 - 1][0] >= 0
            has_marker = False
            head_row = -1
            acc = np.zeros(F)
            for k in range(ipc):
                c, v = s_item[i0 + k]
                if c >= 0:
                    acc = acc + v * B[c]
                elif c == MARKER:
                    if not has_marker and head_partial:
                        H[g] = acc
                        head_row = v
                    else:
                        C[v] = acc
                    has_marker = True
                    acc = np.zeros(F)
            t = s_item[i0 + ipc - 1][0] >= 0
            if t:
                T[g] = acc
            meta.append((has_marker, head_partial, t, head_row))
        for g in range(G):
            head_row = meta[g][3]
            if head_row >= 0:
                j = g - 1
                while j >= 0 and not meta[j][0]:
                    j -= 1
                jf = j if (j >= 0 and meta[j][2]) else j + 1
                from_before = j < 0 and meta[0][1]
                s = np.zeros(F)
                for q in range(jf, g):
                    s = s + T[q]
                s = s + H[g]
                if from_before:
                    part[head[w]] = s
                else:
                    C[head_row] = s
        g = G - 1
        if meta[g][2]:
            j = g
            while j >= 0 and not meta[j][0]:
                j -= 1
            jf = j if (j >= 0 and meta[j][2]) else j + 1
            s = np.zeros(F)
            for q in range(jf, g + 1):
                s = s + T[q]
            part[tail[w]] = s
    for r, sb, se in fix:
        C[r] = part[sb:se + 1].sum(0)
    return C
