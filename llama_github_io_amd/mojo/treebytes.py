"""H2O ``CompressedTree`` byte format (reference: ``hex/genmodel/algos/tree/SharedTreeMojoModel.java``
``scoreTree`` and ``hex/tree/DTree.java`` compression), both directions.

Node: ``nodeType`` u8 | ``colId`` u16 (65535 = the whole tree is one leaf) | ``naSplitDir`` u8 |
split (f32 threshold: left iff x < thr; or a bitset of levels that go RIGHT: ``equal`` = 8 → 4
inline bytes, 12 → u16 bit offset + u32 nbits + bytes) | left-subtree size (``lmask+1`` bytes,
absent when the left child is a leaf) | left subtree | right subtree; a leaf child is an f32.
``nodeType`` bits: 0-1 size-field width-1, 4-5 (48) left is leaf, 2-3 split kind, 6-7 right is leaf.
Little-endian (the writer records ``endianness`` LITTLE_ENDIAN).
"""
from __future__ import annotations

import math
import struct

import numpy as np

NA_VS_REST, NA_LEFT, NA_RIGHT, LEFT, RIGHT = 1, 2, 3, 4, 5


def _node_bytes(t, i, value_map) -> bytes:
    if t.feat[i] < 0:
        return struct.pack("<f", float(value_map(t.value[i])))
    f = int(t.feat[i])
    left, right = int(t.left[i]), int(t.right[i])
    lleaf, rleaf = t.feat[left] < 0, t.feat[right] < 0
    lb = _node_bytes(t, left, value_map)
    rb = _node_bytes(t, right, value_map)
    split = b""
    equal = 0
    if t.is_cat[i]:
        nb = int(t.cat_nbits[i])
        words = t.cat_bits[i]
        goes_left = np.zeros(nb, dtype=bool)
        for lv in range(nb):
            goes_left[lv] = bool((int(words[lv >> 5]) >> (lv & 31)) & 1)
        if goes_left.all():
            nsd = NA_VS_REST
        else:
            nsd = NA_LEFT if t.na_left[i] else NA_RIGHT
            right_bits = ~goes_left
            nbytes = max(1, (nb + 7) // 8)
            bits = np.zeros(nbytes * 8, dtype=np.uint8)
            bits[:nb] = right_bits
            packed = np.packbits(bits, bitorder="little").tobytes()
            equal = 12
            split = struct.pack("<HI", 0, nb) + packed
    else:
        thr = float(t.thr[i])
        if math.isinf(thr) and thr > 0:
            nsd = NA_VS_REST
        else:
            nsd = NA_LEFT if t.na_left[i] else NA_RIGHT
            split = struct.pack("<f", thr)
    node_type = equal
    size_field = b""
    if lleaf:
        node_type |= 48
    else:
        n = len(lb)
        w = 1 if n < (1 << 8) else 2 if n < (1 << 16) else 3 if n < (1 << 24) else 4
        node_type |= (w - 1)
        size_field = n.to_bytes(w, "little")
    if rleaf:
        node_type |= 0xC0
    return struct.pack("<BHB", node_type, f, nsd) + split + size_field + lb + rb


def tree_to_bytes(t, value_map=lambda v: v) -> bytes:
    if t.feat[0] < 0:
        return struct.pack("<BH", 0, 65535) + struct.pack("<f", float(value_map(t.value[0])))
    return _node_bytes(t, 0, value_map)


def bytes_to_tree(buf: bytes, value_map=lambda v: v):
    """Parse a CompressedTree blob into a flat ``ops.forest.Tree``."""
    from ..ops.forest import Tree
    recs = []

    def new():
        recs.append([-1, 0.0, 0, 0, 0, None, 0, -1, -1, 0.0])
        return len(recs) - 1

    def leaf(pos):
        k = new()
        recs[k][9] = value_map(struct.unpack_from("<f", buf, pos)[0])
        return k, pos + 4

    def node(pos):
        nt, col = struct.unpack_from("<BH", buf, pos)
        if col == 65535:
            return leaf(pos + 3)
        nsd = buf[pos + 3]
        pos += 4
        k = new()
        r = recs[k]
        r[0] = col
        equal = nt & 12
        if nsd == NA_VS_REST:
            r[1] = float("inf")
            r[3] = 0
        elif equal == 0:
            r[1] = struct.unpack_from("<f", buf, pos)[0]
            pos += 4
        else:
            if equal == 8:
                off, nbits = 0, 32
                raw = buf[pos:pos + 4]
                pos += 4
            else:
                off, nbits = struct.unpack_from("<HI", buf, pos)
                pos += 6
                nbytes = ((nbits - 1) >> 3) + 1
                raw = buf[pos:pos + nbytes]
                pos += nbytes
            bits = np.unpackbits(np.frombuffer(raw, dtype=np.uint8), bitorder="little")[:nbits].astype(bool)
            nl = off + nbits
            left_levels = np.ones(nl, dtype=bool)
            left_levels[off:off + nbits] = ~bits
            words = np.zeros((nl + 31) // 32, dtype=np.uint32)
            for lv in np.nonzero(left_levels)[0]:
                words[lv >> 5] |= np.uint32(1 << (int(lv) & 31))
            r[4], r[5], r[6] = 1, words, nl
        if nsd != NA_VS_REST:
            r[3] = 1 if nsd in (NA_LEFT, LEFT) else 0
        lmask = nt & 51
        if lmask == 48:
            lk, pos = leaf(pos)
        else:
            w = lmask + 1
            pos += w
            lk, pos = node(pos)
        rk, pos = (leaf(pos) if (nt & 0xC0) == 0xC0 else node(pos))
        recs[k][7], recs[k][8] = lk, rk
        return k, pos

    node(0)
    cols = list(zip(*recs))
    return Tree(feat=np.asarray(cols[0], dtype=np.int32), thr=np.asarray(cols[1], dtype=np.float32),
                bin=np.zeros(len(recs), dtype=np.int32), na_left=np.asarray(cols[3], dtype=np.int8),
                is_cat=np.asarray(cols[4], dtype=np.int8), cat_bits=list(cols[5]),
                cat_nbits=np.asarray(cols[6], dtype=np.int32), left=np.asarray(cols[7], dtype=np.int32),
                right=np.asarray(cols[8], dtype=np.int32), value=np.asarray(cols[9], dtype=np.float32),
                cover=np.zeros(len(recs)), gain=np.zeros(len(recs)))
