#!/usr/bin/env python3
"""blend_export.py -- offline .blend -> scene.json exporter.

Restates the reference's Blender add-on script `Blend/exporter.py` (class Process_objects,
exporter.py:7-277, and its __main__ json.dump(indent=4), :279-295) WITHOUT Blender: the
.blend file is read as data through its own SDNA type catalogue (struct layouts are taken
from the file's DNA1 block, so the reader follows the file's Blender version).  Nothing in
the file is executed.

What the bpy expressions in exporter.py resolve to, and how they are restated here:
  bpy.data.objects            OB blocks in file (= Main list) order
  obj.location / rotation_euler / scale   Object.loc / rot / size (binary32)
  obj.dimensions              |mat4_to_size(object_to_world)| * (mesh bound max - min),
                              binary32 like BKE_object_dimensions_get; object_to_world
                              rebuilt as BKE_object_to_mat4 does (eulO_to_mat3 in double,
                              mul_m3_m3m3 / len_v3 in float) with parent chains
  obj.matrix_world.to_quaternion() @ v   mat3_to_quat (normalize_m3 +
                              mat3_normalized_to_quat_fast) and mul_qt_v3, binary32
  obj.get("velocity"|"aperture"|"focus_dist")   ID properties (IDProperty groups)
  material_slots[0].material  ob->matbits[0] ? ob->mat[0] : mesh->mat[0]
  node.type                   from bNode.idname (ShaderNodeBsdfAnisotropic is Blender 4's
                              Glossy BSDF, type 'BSDF_GLOSSY'; ShaderNodeMix is 'MIX', not
                              'MIX_RGB', exactly as bpy reports it)
  socket.is_linked / links[0] the node tree's bNodeLink list
  image.filepath              Image.name
  light.shadow_soft_size      Lamp.radius;  light.energy = Lamp.energy
  scene.render.resolution_x/y RenderData.xsch / ysch

Usage: blend_export.py FILE.blend [OUT.json]   (stdout when OUT is omitted)
"""
from __future__ import annotations

import json
import math
import os
import re
import struct
import sys
from collections import defaultdict

import numpy as np

f32 = np.float32


# --------------------------------------------------------------------------- SDNA reader
class Blend:
    def __init__(self, path: str):
        self.path = path
        d = open(path, "rb").read()
        if d[:7] != b"BLENDER":
            raise ValueError(f"{path}: not an uncompressed .blend file")
        self.psize = 8 if d[7:8] == b"-" else 4
        self.e = "<" if d[8:9] == b"v" else ">"
        self.version = int(d[9:12])
        self.d = d
        e, ps = self.e, self.psize
        off = 12
        self.blocks = []  # (code, addr, sdna, count, data offset, length)
        hsz = 16 + ps
        while off + hsz <= len(d):
            code = d[off:off + 4]
            ln, = struct.unpack(e + "i", d[off + 4:off + 8])
            addr, = struct.unpack(e + ("Q" if ps == 8 else "I"), d[off + 8:off + 8 + ps])
            sdna, cnt = struct.unpack(e + "ii", d[off + 8 + ps:off + 16 + ps])
            self.blocks.append((code, addr, sdna, cnt, off + hsz, ln))
            off += hsz + ln
            if code == b"ENDB":
                break
        self.by_addr = {b[1]: b for b in self.blocks if b[1]}
        self._sorted = sorted(self.by_addr)
        self._parse_dna()

    def _parse_dna(self):
        d, e = self.d, self.e
        blk = next(b for b in self.blocks if b[0] == b"DNA1")
        p = blk[4]
        p0 = p  # section alignment is relative to the block start

        def align():
            nonlocal p
            p = p0 + ((p - p0 + 3) & ~3)

        def tag(t):
            nonlocal p
            assert d[p:p + 4] == t, t
            p += 4

        def strings():
            nonlocal p
            n, = struct.unpack(e + "i", d[p:p + 4])
            p += 4
            out = []
            for _ in range(n):
                q = d.index(b"\0", p)
                out.append(d[p:q].decode("latin-1"))
                p = q + 1
            align()
            return out

        tag(b"SDNA")
        tag(b"NAME")
        names = strings()
        tag(b"TYPE")
        types = strings()
        tag(b"TLEN")
        tlen = list(struct.unpack(e + "%dh" % len(types), d[p:p + 2 * len(types)]))
        p += 2 * len(types)
        align()
        tag(b"STRC")
        n, = struct.unpack(e + "i", d[p:p + 4])
        p += 4
        self.types, self.tlen = types, tlen
        self.structs = {}   # name -> {field: (offset, type, is_ptr, dims)}
        self.sdna_name = []
        for _ in range(n):
            t, nf = struct.unpack(e + "hh", d[p:p + 4])
            p += 4
            fields, off = {}, 0
            for _ in range(nf):
                ft, fn = struct.unpack(e + "hh", d[p:p + 4])
                p += 4
                raw = names[fn]
                is_ptr = raw.startswith("*") or raw.startswith("(*")
                dims = [int(x) for x in re.findall(r"\[(\d+)\]", raw)]
                base = re.sub(r"\[.*", "", raw).lstrip("*").replace("(", "").replace(")", "")
                count = 1
                for x in dims:
                    count *= x
                size = (self.psize if is_ptr else tlen[ft]) * count
                fields[base] = (off, types[ft], is_ptr, dims)
                off += size
            self.structs[types[t]] = fields
            self.sdna_name.append(types[t])

    # -- values
    def block_at(self, addr: int):
        """(block, byte offset) holding address `addr` (pointers may point inside a block)."""
        if not addr:
            return None, 0
        b = self.by_addr.get(addr)
        if b:
            return b, 0
        import bisect
        i = bisect.bisect_right(self._sorted, addr) - 1
        if i >= 0:
            b = self.by_addr[self._sorted[i]]
            if addr < b[1] + b[5]:
                return b, addr - b[1]
        return None, 0

    def get(self, sname: str, base: int, field: str):
        off, typ, is_ptr, dims = self.structs[sname][field]
        pos = base + off
        e, d = self.e, self.d
        if is_ptr and not dims:
            return struct.unpack(e + ("Q" if self.psize == 8 else "I"), d[pos:pos + self.psize])[0]
        fmt = {"float": "f", "double": "d", "int": "i", "short": "h", "char": "b", "uchar": "B", "int8_t": "b",
               "uint": "I", "ushort": "H", "int64_t": "q", "uint64_t": "Q"}.get(typ)
        if typ in self.structs and not dims:
            return pos  # nested struct: its base offset
        if fmt is None:
            raise KeyError(f"{sname}.{field}: unsupported type {typ}")
        if typ == "char" and dims:
            raw = d[pos:pos + int(np.prod(dims))]
            return raw.split(b"\0", 1)[0].decode("utf-8", "replace")
        if dims:
            cnt = int(np.prod(dims))
            vals = struct.unpack(e + fmt * cnt, d[pos:pos + struct.calcsize(fmt) * cnt])
            return list(vals)
        return struct.unpack(e + fmt, d[pos:pos + struct.calcsize(fmt)])[0]

    def deref(self, addr: int):
        """Absolute file offset of the data at `addr`, or None."""
        b, o = self.block_at(addr)
        return None if b is None else b[4] + o

    def ptr_array(self, addr: int, n: int):
        pos = self.deref(addr)
        if pos is None:
            return []
        fmt = "Q" if self.psize == 8 else "I"
        return list(struct.unpack(self.e + fmt * n, self.d[pos:pos + self.psize * n]))

    def listbase(self, sname_item: str, lb_pos: int):
        """Absolute offsets of the items of a ListBase at file offset lb_pos."""
        out = []
        addr = self.get("ListBase", lb_pos, "first")
        seen = set()
        while addr and addr not in seen:
            seen.add(addr)
            pos = self.deref(addr)
            if pos is None:
                break
            out.append((addr, pos))
            addr = self.get(sname_item, pos, "next")
        return out

    def ids(self, code: bytes):
        return [(b[1], b[4]) for b in self.blocks if b[0] == code]


# --------------------------------------------------------------------------- Blender maths
# eulO_to_mat3 (BLI math_rotation): double trigonometry, result stored as float
_EUL_ORDER = {1: ((0, 1, 2), 0), 2: ((0, 2, 1), 1), 3: ((1, 0, 2), 1), 4: ((1, 2, 0), 0), 5: ((2, 0, 1), 0),
              6: ((2, 1, 0), 1)}


def eulO_to_mat3(e, order):
    (i, j, k), parity = _EUL_ORDER.get(order, _EUL_ORDER[1])
    if parity:
        ti, tj, th = -float(e[i]), -float(e[j]), -float(e[k])
    else:
        ti, tj, th = float(e[i]), float(e[j]), float(e[k])
    ci, cj, ch = math.cos(ti), math.cos(tj), math.cos(th)
    si, sj, sh = math.sin(ti), math.sin(tj), math.sin(th)
    cc, cs, sc, ss = ci * ch, ci * sh, si * ch, si * sh
    M = np.zeros((3, 3), dtype=np.float64)
    M[i][i] = cj * ch
    M[j][i] = sj * sc - cs
    M[k][i] = sj * cc + ss
    M[i][j] = cj * sh
    M[j][j] = sj * ss + cc
    M[k][j] = sj * cs - sc
    M[i][k] = -sj
    M[j][k] = cj * si
    M[k][k] = cj * ci
    if parity:
        M[:, :] = M  # parity handled through the negated angles
    return M.astype(np.float32)  # M[col][row], Blender's column-major float[3][3]


def mul_m3_m3m3(A, B):
    """Blender's mul_m3_m3m3(R, A, B): R[i][j] = B[i][0]*A[0][j] + B[i][1]*A[1][j] + B[i][2]*A[2][j] (float)."""
    R = np.zeros((3, 3), dtype=np.float32)
    for i in range(3):
        for j in range(3):
            R[i][j] = f32(f32(f32(B[i][0] * A[0][j]) + f32(B[i][1] * A[1][j])) + f32(B[i][2] * A[2][j]))
    return R


def mul_m4_m4m4(A, B):
    R = np.zeros((4, 4), dtype=np.float32)
    for i in range(4):
        for j in range(4):
            acc = f32(B[i][0] * A[0][j])
            for k in range(1, 4):
                acc = f32(acc + f32(B[i][k] * A[k][j]))
            R[i][j] = acc
    return R


def len_v3(v):
    return f32(np.sqrt(f32(f32(f32(v[0] * v[0]) + f32(v[1] * v[1])) + f32(v[2] * v[2]))))


def normalize_m3(m):
    """normalize_m3_m3: each column a * (1 / sqrtf(dot(a, a))) in float."""
    out = np.zeros((3, 3), dtype=np.float32)
    for c in range(3):
        a = [f32(x) for x in m[c]]
        d = f32(f32(f32(a[0] * a[0]) + f32(a[1] * a[1])) + f32(a[2] * a[2]))
        if d > f32(1.0e-35):
            inv = f32(f32(1.0) / f32(np.sqrt(d)))
            out[c] = [f32(x * inv) for x in a]
        else:
            out[c] = a
    return out


def quat_from_mat3(m):
    """mat3_to_quat -> mat3_normalized_to_quat_fast (BLI math_rotation, Mike Day's method),
    binary32 throughout; m is Blender's column-major float[3][3]."""
    m = normalize_m3(m)
    one, quarter, two = f32(1.0), f32(0.25), f32(2.0)
    q = [f32(0.0)] * 4
    if m[2][2] < 0.0:
        if m[0][0] > m[1][1]:
            trace = f32(f32(f32(one + m[0][0]) - m[1][1]) - m[2][2])
            s = f32(two * f32(np.sqrt(trace)))
            if m[1][2] < m[2][1]:
                s = -s
            q[1] = f32(quarter * s)
            s = f32(one / s)
            q[0] = f32(f32(m[1][2] - m[2][1]) * s)
            q[2] = f32(f32(m[0][1] + m[1][0]) * s)
            q[3] = f32(f32(m[2][0] + m[0][2]) * s)
            if trace == one and q[0] == 0 and q[2] == 0 and q[3] == 0:
                q[1] = one
        else:
            trace = f32(f32(f32(one - m[0][0]) + m[1][1]) - m[2][2])
            s = f32(two * f32(np.sqrt(trace)))
            if m[2][0] < m[0][2]:
                s = -s
            q[2] = f32(quarter * s)
            s = f32(one / s)
            q[0] = f32(f32(m[2][0] - m[0][2]) * s)
            q[1] = f32(f32(m[0][1] + m[1][0]) * s)
            q[3] = f32(f32(m[1][2] + m[2][1]) * s)
            if trace == one and q[0] == 0 and q[1] == 0 and q[3] == 0:
                q[2] = one
    else:
        if m[0][0] < -m[1][1]:
            trace = f32(f32(f32(one - m[0][0]) - m[1][1]) + m[2][2])
            s = f32(two * f32(np.sqrt(trace)))
            if m[0][1] < m[1][0]:
                s = -s
            q[3] = f32(quarter * s)
            s = f32(one / s)
            q[0] = f32(f32(m[0][1] - m[1][0]) * s)
            q[1] = f32(f32(m[2][0] + m[0][2]) * s)
            q[2] = f32(f32(m[1][2] + m[2][1]) * s)
            if trace == one and q[0] == 0 and q[1] == 0 and q[2] == 0:
                q[3] = one
        else:
            trace = f32(f32(f32(one + m[0][0]) + m[1][1]) + m[2][2])
            s = f32(two * f32(np.sqrt(trace)))
            q[0] = f32(quarter * s)
            s = f32(one / s)
            q[1] = f32(f32(m[1][2] - m[2][1]) * s)
            q[2] = f32(f32(m[2][0] - m[0][2]) * s)
            q[3] = f32(f32(m[0][1] - m[1][0]) * s)
            if trace == one and q[1] == 0 and q[2] == 0 and q[3] == 0:
                q[0] = one
    ln2 = f32(f32(f32(f32(q[0] * q[0]) + f32(q[1] * q[1])) + f32(q[2] * q[2])) + f32(q[3] * q[3]))
    if abs(float(ln2) - 1.0) >= float(f32(0.0002) * f32(3)):
        ln = f32(np.sqrt(ln2))
        q = [f32(x / ln) for x in q]
    return q


def quat_rotate(q, v):
    """mathutils Quaternion @ Vector = mul_qt_v3 (binary32, the C expression order)."""
    q = [f32(t) for t in q]
    r = [f32(t) for t in v]
    t0 = f32(f32(f32(-q[1] * r[0]) - f32(q[2] * r[1])) - f32(q[3] * r[2]))
    t1 = f32(f32(f32(q[0] * r[0]) + f32(q[2] * r[2])) - f32(q[3] * r[1]))
    t2 = f32(f32(f32(q[0] * r[1]) + f32(q[3] * r[0])) - f32(q[1] * r[2]))
    r2 = f32(f32(f32(q[0] * r[2]) + f32(q[1] * r[1])) - f32(q[2] * r[0]))
    r0, r1 = t1, t2
    t1 = f32(f32(f32(f32(t0 * -q[1]) + f32(r0 * q[0])) - f32(r1 * q[3])) + f32(r2 * q[2]))
    t2 = f32(f32(f32(f32(t0 * -q[2]) + f32(r1 * q[0])) - f32(r2 * q[1])) + f32(r0 * q[3]))
    r2 = f32(f32(f32(f32(t0 * -q[3]) + f32(r2 * q[0])) - f32(r0 * q[2])) + f32(r1 * q[1]))
    return [float(t1), float(t2), float(r2)]


# --------------------------------------------------------------------------- the exporter
IDNAME_TYPE = {
    "ShaderNodeBsdfPrincipled": "BSDF_PRINCIPLED", "ShaderNodeBsdfGlass": "BSDF_GLASS",
    "ShaderNodeBsdfDiffuse": "BSDF_DIFFUSE", "ShaderNodeBsdfGlossy": "BSDF_GLOSSY",
    "ShaderNodeBsdfAnisotropic": "BSDF_GLOSSY", "ShaderNodeMixShader": "MIX_SHADER",
    "ShaderNodeTexImage": "TEX_IMAGE", "ShaderNodeMixRGB": "MIX_RGB", "ShaderNodeMix": "MIX",
    "ShaderNodeBump": "BUMP", "ShaderNodeMath": "MATH",
}
OB_MESH, OB_LAMP, OB_CAMERA = 1, 10, 11
LA_LOCAL = 0
IDP_STRING, IDP_INT, IDP_FLOAT, IDP_ARRAY, IDP_GROUP, IDP_DOUBLE = 0, 1, 2, 5, 6, 8


class Exporter:
    def __init__(self, path: str):
        self.B = B = Blend(path)
        self.objects = []
        for addr, pos in B.ids(b"OB\0\0"):
            self.objects.append((addr, pos))
        self._world = {}

    # ---- ID properties (obj.get)
    def idprop(self, id_pos: int, key: str, default):
        B = self.B
        p = B.get("ID", id_pos, "properties")
        gp = B.deref(p)
        if gp is None:
            return default
        grp_data = B.get("IDProperty", gp, "data")
        for _, cp in B.listbase("IDProperty", B.get("IDPropertyData", grp_data, "group")):
            if B.get("IDProperty", cp, "name") != key:
                continue
            t = B.get("IDProperty", cp, "type")
            dp = B.get("IDProperty", cp, "data")
            if t == IDP_INT:
                return B.get("IDPropertyData", dp, "val")
            if t == IDP_FLOAT:
                return float(struct.unpack(B.e + "f", struct.pack(B.e + "i", B.get("IDPropertyData", dp, "val")))[0])
            if t == IDP_DOUBLE:
                lo = B.get("IDPropertyData", dp, "val") & 0xFFFFFFFF
                hi = B.get("IDPropertyData", dp, "val2") & 0xFFFFFFFF
                return struct.unpack("<d", struct.pack("<II", lo, hi))[0]
            if t == IDP_ARRAY:
                n = B.get("IDProperty", cp, "len")
                sub = B.get("IDProperty", cp, "subtype")
                arr = B.deref(B.get("IDPropertyData", dp, "pointer"))
                fmt = {IDP_FLOAT: "f", IDP_DOUBLE: "d", IDP_INT: "i"}[sub]
                return [float(x) if fmt != "i" else x for x in
                        struct.unpack(B.e + fmt * n, B.d[arr:arr + struct.calcsize(fmt) * n])]
            return default
        return default

    # ---- object transforms
    def local_mat4(self, pos):
        B = self.B
        loc = np.array(B.get("Object", pos, "loc"), dtype=np.float32)
        dloc = np.array(B.get("Object", pos, "dloc"), dtype=np.float32)
        size = np.array(B.get("Object", pos, "size"), dtype=np.float32)
        dscale = np.array(B.get("Object", pos, "dscale"), dtype=np.float32)
        rot = B.get("Object", pos, "rot")
        drot = B.get("Object", pos, "drot")
        rotmode = B.get("Object", pos, "rotmode")
        if rotmode < 1 or rotmode > 6:
            raise NotImplementedError(f"rotation mode {rotmode} (quaternion / axis-angle) not restated")
        smat = np.diag((size * dscale).astype(np.float32))
        rmat = eulO_to_mat3(rot, rotmode)
        dmat = eulO_to_mat3(drot, rotmode)
        rmat = mul_m3_m3m3(dmat, rmat)
        tmat = mul_m3_m3m3(rmat, smat)
        M = np.zeros((4, 4), dtype=np.float32)
        M[:3, :3] = tmat
        M[3, :3] = (loc + dloc).astype(np.float32)
        M[3, 3] = 1.0
        return M

    def world_mat4(self, addr, pos):
        if addr in self._world:
            return self._world[addr]
        B = self.B
        M = self.local_mat4(pos)
        par = B.get("Object", pos, "parent")
        if par:
            ppos = B.deref(par)
            pinv = np.array(B.get("Object", pos, "parentinv"), dtype=np.float32).reshape(4, 4)
            M = mul_m4_m4m4(mul_m4_m4m4(self.world_mat4(par, ppos), pinv), M)
        self._world[addr] = M
        return M

    def mesh_bounds(self, me_pos):
        B = self.B
        n = B.get("Mesh", me_pos, "totvert")
        vd = B.get("Mesh", me_pos, "vdata")
        layers = B.deref(B.get("CustomData", vd, "layers"))
        tot = B.get("CustomData", vd, "totlayer")
        pts = None
        lsz = B.tlen[B.types.index("CustomDataLayer")]
        for li in range(tot):
            lp = layers + li * lsz
            if B.get("CustomDataLayer", lp, "name") == "position":
                dp = B.deref(B.get("CustomDataLayer", lp, "data"))
                pts = np.frombuffer(B.d, dtype=B.e + "f4", count=3 * n, offset=dp).reshape(n, 3)
        if pts is None:
            raise NotImplementedError("mesh without a 'position' vertex layer")
        return pts.min(0).astype(np.float32), pts.max(0).astype(np.float32)

    def dimensions(self, addr, pos):
        B = self.B
        lo, hi = self.mesh_bounds(B.deref(B.get("Object", pos, "data")))
        M = self.world_mat4(addr, pos)
        scale = [len_v3(M[c][:3]) for c in range(3)]
        return [float(f32(abs(scale[a]) * f32(hi[a] - lo[a]))) for a in range(3)]

    # ---- materials / node trees (exporter.py:12-170)
    def material(self, ob_pos):
        B = self.B
        data = {
            'diffuse_color': [0.8, 0.8, 0.8], 'specular_color': [0.0, 0.0, 0.0], 'roughness': 0.5,
            'k_ambient': 0.1, 'k_diffuse': 0.9, 'k_specular': 0.3, 'reflectivity': 0.0, 'transparency': 0.0,
            'refractive_index': 1.0, 'texture_file': "",
        }
        totcol = B.get("Object", ob_pos, "totcol")
        if totcol <= 0:
            return data
        matbits = B.deref(B.get("Object", ob_pos, "matbits"))
        use_ob = matbits is not None and B.d[matbits] != 0
        if use_ob:
            ma = B.ptr_array(B.get("Object", ob_pos, "mat"), 1)
        else:
            me = B.deref(B.get("Object", ob_pos, "data"))
            ma = B.ptr_array(B.get("Mesh", me, "mat"), 1) if me is not None else []
        ma_pos = B.deref(ma[0]) if ma and ma[0] else None
        if ma_pos is None:
            return data
        nt = B.deref(B.get("Material", ma_pos, "nodetree"))
        if nt is None:
            return data
        nodes = [p for _, p in B.listbase("bNode", B.get("bNodeTree", nt, "nodes"))]
        node_addr = {p: a for a, p in B.listbase("bNode", B.get("bNodeTree", nt, "nodes"))}
        links = [p for _, p in B.listbase("bNodeLink", B.get("bNodeTree", nt, "links"))]
        addr_pos = {a: p for p, a in node_addr.items()}

        def ntype(n):
            return IDNAME_TYPE.get(B.get("bNode", n, "idname"), B.get("bNode", n, "idname"))

        def inputs(n):
            return [(a, p) for a, p in B.listbase("bNodeSocket", B.get("bNode", n, "inputs"))]

        def sock(n, key):
            if isinstance(key, int):
                ins = inputs(n)
                return ins[key] if key < len(ins) else None
            for a, p in inputs(n):
                if B.get("bNodeSocket", p, "name") == key:
                    return a, p
            return None

        def has(n, key):
            return sock(n, key) is not None

        def sock_links(s):
            return [l for l in links if B.get("bNodeLink", l, "tosock") == s[0]]

        def default(s):
            dv = B.deref(B.get("bNodeSocket", s[1], "default_value"))
            idn = B.get("bNodeSocket", s[1], "idname")
            if "Color" in idn:
                return [float(x) for x in struct.unpack(B.e + "4f", B.d[dv:dv + 16])]
            if "Float" in idn:
                return float(struct.unpack(B.e + "f", B.d[dv + 4:dv + 8])[0])
            raise NotImplementedError(idn)

        def from_node(l):
            return addr_pos[B.get("bNodeLink", l, "fromnode")]

        def get_input_color(n, name):
            s = sock(n, name)
            if s is not None:
                return default(s)[:3]
            return [1.0, 1.0, 1.0]

        def find_texture_recursive(s):
            ls = sock_links(s)
            if not ls:
                return ""
            fn = from_node(ls[0])
            t = ntype(fn)
            if t == 'TEX_IMAGE':
                im = B.deref(B.get("bNode", fn, "id"))
                if im is not None:
                    return os.path.basename(B.get("Image", im, "name"))
            if t == 'BUMP':
                h = sock(fn, 'Height')
                if sock_links(h):
                    return find_texture_recursive(h)
            if t in ['MIX_RGB', 'MATH', 'MIX_SHADER']:
                ins = inputs(fn)
                for idx in range(min(2, len(ins))):
                    found = find_texture_recursive(ins[idx])
                    if found:
                        return found
            return ""

        def find_tint_color(s):
            ls = sock_links(s)
            if not ls:
                return default(s)[:3]
            fn = from_node(ls[0])
            if ntype(fn) == 'MIX_RGB':
                c1, c2 = sock(fn, 1), sock(fn, 2)
                c1l, c2l = bool(sock_links(c1)), bool(sock_links(c2))
                if c1l and not c2l:
                    return default(c2)[:3]
                if c2l and not c1l:
                    return default(c1)[:3]
            return [1.0, 1.0, 1.0]

        principled = next((n for n in nodes if ntype(n) == 'BSDF_PRINCIPLED'), None)
        if principled is not None:
            bc = sock(principled, 'Base Color')
            data['diffuse_color'] = find_tint_color(bc)
            if not sock_links(bc):
                data['diffuse_color'] = default(bc)[:3]
            data['roughness'] = default(sock(principled, 'Roughness'))
            data['reflectivity'] = default(sock(principled, 'Metallic'))
            if has(principled, 'Transmission Weight'):
                data['transparency'] = default(sock(principled, 'Transmission Weight'))
            elif has(principled, 'Transmission'):
                data['transparency'] = default(sock(principled, 'Transmission'))
            if has(principled, 'IOR'):
                data['refractive_index'] = default(sock(principled, 'IOR'))
            data['texture_file'] = find_texture_recursive(bc)
            return data

        glass = next((n for n in nodes if ntype(n) == 'BSDF_GLASS'), None)
        if glass is not None:
            data['diffuse_color'] = get_input_color(glass, 'Color')
            data['specular_color'] = [1.0, 1.0, 1.0]
            data['transparency'] = 1.0
            data['refractive_index'] = default(sock(glass, 'IOR'))
            data['roughness'] = default(sock(glass, 'Roughness'))
            return data

        diffuse = next((n for n in nodes if ntype(n) == 'BSDF_DIFFUSE'), None)
        glossy = next((n for n in nodes if ntype(n) == 'BSDF_GLOSSY'), None)
        mix = next((n for n in nodes if ntype(n) == 'MIX_SHADER'), None)
        if diffuse is not None:
            data['texture_file'] = find_texture_recursive(sock(diffuse, 'Color'))
            if not data['texture_file'] and sock_links(sock(diffuse, 'Normal')):
                data['texture_file'] = find_texture_recursive(sock(diffuse, 'Normal'))
            data['diffuse_color'] = find_tint_color(sock(diffuse, 'Color'))
        if glossy is not None:
            data['specular_color'] = get_input_color(glossy, 'Color')
            data['roughness'] = default(sock(glossy, 'Roughness'))
            if mix is not None:
                fac = default(sock(mix, 'Fac'))
                is_glossy_top = False
                mins = inputs(mix)
                if len(mins) > 1:
                    for l in sock_links(mins[1]):
                        if from_node(l) == glossy:
                            is_glossy_top = True
                            break
                if is_glossy_top:
                    k_spec, k_diff = 1.0 - fac, fac
                else:
                    k_spec, k_diff = fac, 1.0 - fac
                data['k_specular'] = k_spec
                data['k_diffuse'] = k_diff
                data['reflectivity'] = k_spec
            else:
                data['k_specular'] = 1.0
                data['k_diffuse'] = 0.0
                data['reflectivity'] = 1.0
        return data

    # ---- Process_objects.process (exporter.py:172-277)
    def process(self) -> dict:
        B = self.B
        out = defaultdict(list)
        for addr, pos in self.objects:
            idp = B.get("Object", pos, "id")
            name = B.get("ID", idp, "name")[2:]
            typ = B.get("Object", pos, "type")
            loc = [float(x) for x in B.get("Object", pos, "loc")]
            rot = [float(x) for x in B.get("Object", pos, "rot")]
            if typ == OB_MESH:
                mat = self.material(pos)
                if 'Sphere' in name:
                    dims = self.dimensions(addr, pos)
                    out['spheres'].append({
                        'location': loc, 'rotation': rot, 'scale': [dims[0] / 2.0, dims[1] / 2.0, dims[2] / 2.0],
                        'velocity': list(self.idprop(idp, "velocity", [0.0, 0.0, 0.0])), 'material': mat})
                elif 'Cube' in name:
                    dims = self.dimensions(addr, pos)
                    out['cubes'].append({'translation': loc, 'rotation': rot, 'scale': [dims[0], dims[1], dims[2]],
                                         'material': mat})
                elif 'Plane' in name:
                    dims = self.dimensions(addr, pos)
                    out['rectangles'].append({'translation': loc, 'rotation': rot,
                                              'scale': [dims[0], dims[1], 1.0], 'material': mat})
            elif typ == OB_CAMERA:
                ca = B.deref(B.get("Object", pos, "data"))
                M = self.world_mat4(addr, pos)
                q = quat_from_mat3(M[:3, :3])
                dof = B.get("Camera", ca, "dof")
                out['cameras'].append({
                    'location': loc,
                    'gaze_vector': quat_rotate(q, (0.0, 0.0, -1.0)),
                    'focal_length': float(B.get("Camera", ca, "lens")),
                    'sensor_width': float(B.get("Camera", ca, "sensor_x")),
                    'sensor_height': float(B.get("Camera", ca, "sensor_y")),
                    'up_vector': quat_rotate(q, (0.0, 1.0, 0.0)),
                    'aperture': self.idprop(idp, "aperture", 0.0),
                    'focus_dist': self.idprop(idp, "focus_dist",
                                              float(B.get("CameraDOFSettings", dof, "focus_distance"))),
                })
            elif typ == OB_LAMP:
                la = B.deref(B.get("Object", pos, "data"))
                if B.get("Lamp", la, "type") == LA_LOCAL:
                    out['lights'].append({
                        'location': loc, 'intensity': float(B.get("Lamp", la, "energy")),
                        'color': [float(B.get("Lamp", la, c)) for c in ("r", "g", "b")],
                        'radius': float(B.get("Lamp", la, "radius")),
                    })
        sc = B.ids(b"SC\0\0")[0][1]
        r = B.get("Scene", sc, "r")
        out['render'] = {'resolution_x': B.get("RenderData", r, "xsch"),
                         'resolution_y': B.get("RenderData", r, "ysch")}
        return out


def export(path: str) -> str:
    return json.dumps(Exporter(path).process(), indent=4)


def main():
    if len(sys.argv) < 2:
        print(__doc__)
        sys.exit(2)
    txt = export(sys.argv[1])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(txt)
    else:
        print(txt)


if __name__ == "__main__":
    main()
