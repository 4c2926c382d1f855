"""Generate tests/golden/mpi_h_constants.json: every integer-valued #define of
the reference's public header (src/include/mpi.h), as the x64 build sees it
(_WIN64 defined, the SAL and C++ branches off).  Run in the survey container
only, where /root/reference exists:

    python tests/golden/gen_mpi_h_constants.py /root/reference/src/include/mpi.h

The output is data (name -> value), not header text; tests/test_abi.py checks
include/mpi.h against it so the ABI cannot drift."""
import json
import os
import re
import sys

CAST = re.compile(r"\(\s*(?:MPI_\w+|int|unsigned|unsigned int|long|long long)\s*\)")


def evaluate(expr, known):
    e = CAST.sub("", expr).strip()
    if not e or '"' in e or "void" in e or "*" in e:
        return None
    e = re.sub(r"\b(0x[0-9a-fA-F]+|\d+)[uUlL]+\b", r"\1", e)
    names = re.findall(r"\b[A-Za-z_]\w*", e)
    for n in names:
        if n not in known:
            return None
    try:
        v = eval(e, {"__builtins__": {}}, dict(known))
    except Exception:
        return None
    return int(v) if isinstance(v, int) else None


def parse(text, defined):
    out, known, stack = {}, {}, []           # stack of (taking, any_taken)
    def cond(expr):
        expr = expr.strip()
        expr = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if m.group(1) in defined or m.group(1) in known else "0", expr)
        expr = expr.replace("!", " not ").replace("&&", " and ").replace("||", " or ")
        for n in re.findall(r"[A-Za-z_]\w*", expr):
            if n not in ("not", "and", "or"):
                expr = re.sub(rf"\b{n}\b", str(known.get(n, 0)), expr)
        try:
            return bool(eval(expr, {"__builtins__": {}}, {}))
        except Exception:
            return False
    for raw in text.splitlines():
        line = raw.split("//")[0].strip()
        taking = all(t for t, _ in stack)
        m = re.match(r"#\s*(ifdef|ifndef|if|elif|else|endif)\b(.*)", line)
        if m:
            kw, rest = m.group(1), m.group(2).strip()
            if kw in ("ifdef", "ifndef"):
                d = rest.split()[0] in defined or rest.split()[0] in known
                t = d if kw == "ifdef" else not d
                stack.append((t, t))
            elif kw == "if":
                t = cond(rest)
                stack.append((t, t))
            elif kw == "elif":
                _, anyt = stack.pop()
                t = (not anyt) and cond(rest)
                stack.append((t, anyt or t))
            elif kw == "else":
                _, anyt = stack.pop()
                stack.append((not anyt, True))
            else:
                stack.pop()
            continue
        if not taking:
            continue
        m = re.match(r"#\s*define\s+(\w+)\s+(.+)$", line)
        if m:
            name, val = m.group(1), m.group(2).split("/*")[0].strip()
            v = evaluate(val, known)
            if v is not None:
                known[name] = v
                out[name] = v
    return out


if __name__ == "__main__":
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/include/mpi.h"
    with open(src, encoding="utf-8", errors="replace") as f:
        consts = parse(f.read(), defined={"_WIN64", "MSMPI_NO_SAL"})
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mpi_h_constants.json")
    with open(dst, "w") as f:
        json.dump({"source": "src/include/mpi.h (x64: _WIN64 defined)", "constants": consts}, f, indent=0,
                  sort_keys=True)
    print(len(consts), "constants ->", dst)
