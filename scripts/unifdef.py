#!/usr/bin/env python3
"""Minimal unifdef: rewrite sources as if the given macros were undefined.

Handles #ifdef / #ifndef / #if [!]defined(X) [&&|| ...] / #elif / #else / #endif whose
conditions mention only the listed macros; other conditionals pass through untouched (a
condition mixing listed and unlisted macros is an error). Used to strip timing-experiment
variants from the product kernels.

usage: unifdef.py FILE MACRO [MACRO ...]
"""
import re
import sys


def cond_value(expr, undef):
    names = set(re.findall(r"defined\s*\(\s*(\w+)\s*\)", expr))
    if not names or not names & undef:
        return None
    if names - undef:
        raise SystemExit(f"mixed condition: {expr!r}")
    py = re.sub(r"defined\s*\(\s*\w+\s*\)", "False", expr)
    py = py.replace("&&", " and ").replace("||", " or ")
    py = re.sub(r"!(?!=)", " not ", py)
    return bool(eval(py))


def main():
    path, undef = sys.argv[1], set(sys.argv[2:])
    out = []
    # stack entries: [managed, emitting_now, any_taken, parent_emitting]
    stack = []
    emitting = True
    for line in open(path).read().split("\n"):
        s = line.strip()
        m = re.match(r"#\s*(ifdef|ifndef|if|elif|else|endif)\b(.*)", s)
        if not m:
            if emitting:
                out.append(line)
            continue
        kw, rest = m.group(1), re.sub(r"//.*", "", m.group(2)).strip()
        if kw in ("ifdef", "ifndef", "if"):
            if kw == "ifdef":
                expr = f"defined({rest})"
            elif kw == "ifndef":
                expr = f"!defined({rest})"
            else:
                expr = rest
            v = cond_value(expr, undef)
            if v is None:
                stack.append([False, emitting, False, emitting])
                if emitting:
                    out.append(line)
            else:
                stack.append([True, emitting and v, v, emitting])
                emitting = emitting and v
        elif kw == "elif":
            top = stack[-1]
            if not top[0]:
                v = cond_value(rest, undef)
                if v is not None:
                    raise SystemExit(f"managed #elif under unmanaged #if: {line!r}")
                if top[3]:
                    out.append(line)
                continue
            v = cond_value(rest, undef)
            if v is None:
                raise SystemExit(f"unmanaged #elif under managed #if: {line!r}")
            take = v and not top[2]
            top[2] = top[2] or v
            emitting = top[3] and take
        elif kw == "else":
            top = stack[-1]
            if not top[0]:
                if top[3]:
                    out.append(line)
                continue
            emitting = top[3] and not top[2]
            top[2] = True
        else:  # endif
            top = stack.pop()
            emitting = top[3]
            if not top[0] and emitting:
                out.append(line)
    assert not stack, "unbalanced conditionals"
    open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    main()
