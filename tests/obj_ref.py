"""Test-side restatement of OBJ.Load (OBJ.cs:11-165) in plain Python, the checker for
the native pt_obj_load.  Follows the reference line by line: ToLower + Split(' ')
(OBJ.cs:33-35), the dummy normal (:18), Split({"//","/"}, RemoveEmptyEntries) (:89-101),
fan triangulation (:110-113), Triangle.FixNormals (Triangle.cs:199-204, 224-237)."""
import numpy as np

f32 = np.float32


def _normalize(v):
    x, y, z = (f32(c) for c in v)
    ln = np.sqrt(f32(f32(x * x + y * y) + z * z), dtype=np.float32)
    return (f32(x / ln), f32(y / ln), f32(z / ln))


def _face_normal(a, b, c):
    e1 = tuple(f32(b[i] - a[i]) for i in range(3))
    e2 = tuple(f32(c[i] - a[i]) for i in range(3))
    cr = (f32(e1[1] * e2[2] - e1[2] * e2[1]), f32(e1[2] * e2[0] - e1[0] * e2[2]), f32(e1[0] * e2[1] - e1[1] * e2[0]))
    return _normalize(cr)


def _split_slashes(s):
    out, cur, i = [], "", 0
    while i < len(s):
        if s[i] == "/":
            if cur:
                out.append(cur)
            cur = ""
            i += 2 if s[i:i + 2] == "//" else 1
        else:
            cur += s[i]
            i += 1
    if cur:
        out.append(cur)
    return out


def load(path):
    vs, vts, vns = [], [], [(f32(0), f32(0), f32(0))]
    tri = {k: [] for k in ("v1", "v2", "v3", "n1", "n2", "n3", "t1", "t2", "t3")}
    with open(path, "rb") as fh:
        text = fh.read().decode("latin-1")
    for line in text.replace("\r\n", "\n").replace("\r", "\n").split("\n"):
        words = [w for w in line.lower().split(" ") if w != ""]
        if not words:
            continue
        typ, words = words[0], words[1:]
        if typ == "v":
            vs.append(tuple(f32(float(w)) for w in words[:3]))
        elif typ == "vt":
            vts.append((f32(float(words[0])), f32(float(words[1])), f32(0)))
        elif typ == "vn":
            vns.append(tuple(f32(float(w)) for w in words[:3]))
        elif typ == "f":
            n = len(words)
            fv, ft, fn = [0] * n, [0] * n, [0] * n
            for c, arg in enumerate(words):
                p = _split_slashes(arg)
                if len(p) > 0:
                    fv[c] = int(p[0]) - 1
                if len(p) > 1:
                    ft[c] = int(p[1]) - 1
                if len(p) > 2:
                    fn[c] = int(p[2]) - 1
            for i in range(1, n - 1):
                idx = (0, i, i + 1)
                zero = (f32(0), f32(0), f32(0))
                V = [vs[fv[k]] if vs else zero for k in idx]
                T = [vts[ft[k]] if vts else zero for k in idx]
                N = [vns[fn[k]] for k in idx]
                face = _face_normal(*V)
                N = [face if all(c == 0 for c in nn) else nn for nn in N]
                for j, k in enumerate(("1", "2", "3")):
                    tri["v" + k].append(V[j])
                    tri["n" + k].append(N[j])
                    tri["t" + k].append(T[j])
    return {k: np.array(v, np.float32).reshape(-1, 3) for k, v in tri.items()}
