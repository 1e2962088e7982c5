"""Extract the schema, attributes and data of the reference's CDL fixture
src/utils/ncmpigen/c0.cdl into tests/golden/c0_cdl.json (data only: names,
types, shapes and the literal values, each typed as CDL types it: `b` byte,
`s` short, plain integer int, `f` float, other reals double, strings text).

    python tests/golden/make_c0.py /root/reference/src/utils/ncmpigen/c0.cdl

Run once in the build container; the JSON is what the tests read (the
reference tree does not exist on the GPU box).  The parser covers the CDL
subset c0.cdl uses: `//` comments, UNLIMITED, quoted strings with C escapes
(octal and \\t), numeric suffixes b/s/f, multi-line data lists.
"""
import json
import re
import sys

TYPES = {"char": 2, "byte": 1, "short": 3, "int": 4, "float": 5, "double": 6}


def unescape(s):
    out, i = bytearray(), 0
    while i < len(s):
        c = s[i]
        if c != "\\":
            out += c.encode("latin1")
            i += 1
            continue
        n = s[i + 1]
        if n in "01234567":
            j = i + 1
            while j < len(s) and j < i + 4 and s[j] in "01234567":
                j += 1
            out.append(int(s[i + 1:j], 8) & 0xFF)
            i = j
        else:
            out += {"t": b"\t", "n": b"\n", "\\": b"\\", '"': b'"', "'": b"'"}[n]
            i += 2
    return bytes(out)


TOKEN = re.compile(r'"((?:[^"\\]|\\.)*)"|([^,\s;]+)')


def values(text):
    """a CDL value list -> (xtype, [values]) or ("text", [bytes per string])"""
    strs, nums = [], []
    for m in TOKEN.finditer(text):
        if m.group(1) is not None:
            strs.append(unescape(m.group(1)))
        else:
            nums.append(m.group(2))
    if strs:
        return 2, strs
    xt, vals = None, []
    for t in nums:
        if t[-1] in "bB":
            t_xt, v = 1, int(t[:-1])
        elif t[-1] in "sS":
            t_xt, v = 3, int(t[:-1])
        elif t[-1] in "fF" and not t.lower().startswith("0x"):
            t_xt, v = 5, float(t[:-1])
        elif re.fullmatch(r"[+-]?\d+", t):
            t_xt, v = 4, int(t)
        else:
            t_xt, v = 6, float(t)
        xt = t_xt if xt is None else xt
        vals.append(v)
    return xt, vals


def main(path, out):
    src = "\n".join(line.split("//")[0] for line in open(path, encoding="latin1").read().split("\n"))
    body = src[src.index("{") + 1:src.rindex("}")]
    dims_s = body[body.index("dimensions:") + len("dimensions:"):body.index("variables:")]
    vars_s = body[body.index("variables:") + len("variables:"):body.index("data:")]
    data_s = body[body.index("data:") + len("data:"):]
    dims = []
    for st in dims_s.split(";"):
        st = st.strip()
        if st:
            name, ln = [x.strip() for x in st.split("=")]
            dims.append([name, 0 if ln == "UNLIMITED" else int(ln)])
    dnames = [d[0] for d in dims]
    variables, atts = [], []
    for st in vars_s.split(";"):
        st = st.strip()
        if not st:
            continue
        m = re.match(r"(char|byte|short|int|float|double)\s+([^\s(]+)\s*(?:\(([^)]*)\))?$", st)
        if m:
            ds = [dnames.index(x.strip()) for x in m.group(3).split(",")] if m.group(3) else []
            variables.append({"name": m.group(2), "xtype": TYPES[m.group(1)], "dims": ds})
            continue
        lhs, rhs = st.split("=", 1)
        var, att = lhs.strip().split(":", 1)
        xt, vals = values(rhs)
        atts.append({"var": var.strip(), "name": att.strip(), "xtype": xt,
                     "values": [v.decode("latin1") for v in vals] if xt == 2 else vals})
    data = {}
    for st in data_s.split(";"):
        st = st.strip()
        if not st:
            continue
        lhs, rhs = st.split("=", 1)
        xt, vals = values(rhs)
        data[lhs.strip()] = {"text": [v.decode("latin1") for v in vals]} if xt == 2 else {"numbers": vals}
    json.dump({"source": "src/utils/ncmpigen/c0.cdl (PnetCDF 1.15.0)", "dims": dims, "vars": variables,
               "atts": atts, "data": data}, open(out, "w"), indent=0)


if __name__ == "__main__":
    import os
    main(sys.argv[1], os.path.join(os.path.dirname(os.path.abspath(__file__)), "c0_cdl.json"))
