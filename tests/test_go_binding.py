"""CPU guard for the Go binding (integration/go/**): there is no Go toolchain in
this image, so a lexer checks what `go build` would reject first.

The binding is the cgo package a maintainer drops in beside the reference's
sketch aggregator (internal/engine/impl/sketch/task.go:1,21-65, registered as
task_factory.go:24 does).  For every .go file:
  - the first token outside comments is `package sketchgpu`;
  - at top level every line starts a declaration (import/func/var/const/type),
    so stray text between declarations fails;
  - (), [] and {} balance outside strings, runes and comments;
  - every C.gns_* the file calls is a function include/gns_sketch.h declares,
    called with the declared number of arguments, and every C.GNS_* / C.gns_*
    name used as a value or type is declared there too.
"""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO_FILES = sorted(glob.glob(os.path.join(ROOT, "integration", "go", "**", "*.go"), recursive=True))

_TOP = {"package", "import", "func", "var", "const", "type"}
_OPEN = {"(": ")", "[": "]", "{": "}"}
_CLOSE = {v: k for k, v in _OPEN.items()}


def go_tokens(src):
    """Yield (kind, text, line) for Go source: kinds 'id', 'punct', 'str',
    'num'.  Comments are dropped; raw strings, interpreted strings and runes are
    single tokens.  Raises ValueError on an unterminated literal or comment."""
    i, n, line = 0, len(src), 1
    while i < n:
        c = src[i]
        if c == "\n":
            line += 1
            i += 1
        elif c in " \t\r":
            i += 1
        elif src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            if j < 0:
                raise ValueError(f"line {line}: unterminated comment")
            line += src.count("\n", i, j)
            i = j + 2
        elif c == "`":
            j = src.find("`", i + 1)
            if j < 0:
                raise ValueError(f"line {line}: unterminated raw string")
            yield "str", src[i:j + 1], line
            line += src.count("\n", i, j)
            i = j + 1
        elif c in "\"'":
            j = i + 1
            while j < n and src[j] != c:
                if src[j] == "\n":
                    raise ValueError(f"line {line}: newline in literal")
                j += 2 if src[j] == "\\" else 1
            if j >= n:
                raise ValueError(f"line {line}: unterminated literal")
            yield "str", src[i:j + 1], line
            i = j + 1
        elif c.isalpha() or c == "_":
            m = re.compile(r"[A-Za-z_0-9]+").match(src, i)
            yield "id", m.group(0), line
            i = m.end()
        elif c.isdigit():
            m = re.compile(r"[0-9A-Za-z_.]+").match(src, i)
            yield "num", m.group(0), line
            i = m.end()
        else:
            yield "punct", c, line
            i += 1


def header_decls():
    """Function name -> parameter count, and every other gns_/GNS_ name, from
    include/gns_sketch.h (comments stripped)."""
    txt = open(os.path.join(ROOT, "include", "gns_sketch.h")).read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", " ", txt)
    funcs = {}
    for m in re.finditer(r"\b(gns_[a-z0-9_]+)\s*\(([^()]*)\)\s*;", txt):
        params = m.group(2).strip()
        funcs[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    names = set(re.findall(r"\b((?:gns|GNS)_[A-Za-z0-9_]+)\b", txt))
    return funcs, names


def check_go_file(src):
    """Return a list of problems (empty when the file passes)."""
    problems = []
    try:
        toks = list(go_tokens(src))
    except ValueError as e:
        return [str(e)]
    if len(toks) < 2 or toks[0][1] != "package" or toks[1][1] != "sketchgpu":
        first = " ".join(t[1] for t in toks[:2])
        problems.append(f"first tokens are {first!r}, not 'package sketchgpu'")
    stack, last_line = [], 0
    for kind, text, line in toks:
        if line != last_line and not stack and not (kind == "punct" and text in _CLOSE):
            if not (kind == "id" and text in _TOP):
                problems.append(f"line {line}: top-level line starts with {text!r}")
        last_line = line
        if kind == "punct" and text in _OPEN:
            stack.append((text, line))
        elif kind == "punct" and text in _CLOSE:
            if not stack or stack[-1][0] != _CLOSE[text]:
                problems.append(f"line {line}: unbalanced {text!r}")
                return problems
            stack.pop()
    if stack:
        problems.append(f"unclosed {stack[-1][0]!r} from line {stack[-1][1]}")
        return problems

    funcs, names = header_decls()
    for i, (kind, text, line) in enumerate(toks):
        if not (kind == "id" and text == "C" and i + 2 < len(toks) and toks[i + 1][1] == "."):
            continue
        name = toks[i + 2][1]
        if not re.match(r"(gns|GNS)_", name):
            continue  # C.uint32_t, C.GoString, C.free ...
        is_call = i + 3 < len(toks) and toks[i + 3][1] == "("
        if is_call and name in funcs:
            depth, args, j, empty = 0, 1, i + 4, True
            while True:
                t = toks[j][1] if toks[j][0] == "punct" else None
                if t in _OPEN:
                    depth += 1
                elif t in _CLOSE:
                    if depth == 0:
                        break
                    depth -= 1
                elif t == "," and depth == 0:
                    args += 1
                if not (toks[j][0] == "punct" and toks[j][1] == ")" and depth == 0):
                    empty = False
                j += 1
            got = 0 if empty else args
            if got != funcs[name]:
                problems.append(f"line {line}: C.{name} called with {got} args, header declares {funcs[name]}")
        elif name not in names:
            problems.append(f"line {line}: C.{name} is not declared in include/gns_sketch.h")
    return problems


def test_go_files_present():
    names = {os.path.basename(p) for p in GO_FILES}
    assert {"sketchgpu.go", "task.go"} <= names, names


@pytest.mark.parametrize("path", GO_FILES, ids=lambda p: os.path.relpath(p, ROOT))
def test_go_file_lexes(path):
    problems = check_go_file(open(path).read())
    assert not problems, problems


def test_checker_catches_round5_breakage():
    """The round-5 regression: the package clause replaced by a stray line."""
    good = 'package sketchgpu\n\nimport (\n\t"fmt"\n)\n\nfunc f() { fmt.Println("x") }\n'
    assert check_go_file(good) == []
    bad = '// header\n\ntoolchain there).\n\nimport (\n\t"fmt"\n)\n\nfunc f() { fmt.Println("x") }\n'
    probs = check_go_file(bad)
    assert any("package sketchgpu" in p for p in probs), probs
    assert any("unbalanced" in p or "top-level" in p for p in probs), probs
    assert check_go_file("package sketchgpu\nfunc f() { a := []int{1, 2}\n") != []
    assert check_go_file('package sketchgpu\nvar s = "a(b"\nvar r = \'(\'\nvar q = `)`\n') == []


def test_checker_catches_cgo_arity():
    src = ('package sketchgpu\n/*\n#include "gns_sketch.h"\n*/\nimport "C"\n'
           'func f(h *C.gns_cm) { C.gns_cm_flush(h, 1) }\n')
    probs = check_go_file(src)
    assert any("C.gns_cm_flush called with 2 args" in p for p in probs), probs
    assert check_go_file(src.replace("C.gns_cm_flush(h, 1)", "C.gns_cm_flush(h)")) == []
    probs = check_go_file(src.replace("C.gns_cm_flush(h, 1)", "C.gns_no_such(h)"))
    assert any("gns_no_such" in p for p in probs), probs
