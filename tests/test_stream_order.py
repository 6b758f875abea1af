"""Every device-memory write of the C ABI is ordered on one of the handle's streams.

The handle's streams are created with hipStreamNonBlocking, so they do not wait for the null
stream: a synchronous hipMemcpy / hipMemset (null stream) into a buffer that enqueued or
pipelined work reads or writes is unordered with that work (round 4: a partials buffer zeroed by
a null-stream hipMemset after a fresh handle's first counting decode had stored into it).  This
test reads the native sources and fails on any synchronous copy or fill outside pscl_create
(where no work has been enqueued yet).  CPU only: source analysis, no GPU.
"""
import re
from pathlib import Path

CSRC = Path(__file__).resolve().parent.parent / "polar_code_amd" / "csrc"
SYNC_CALLS = re.compile(r"\b(hipMemcpy|hipMemset|hipMemcpyToSymbol|hipMemcpyHtoD|hipMemcpyDtoH|hipMemcpyDtoD|"
                        r"hipMemsetD8|hipMemsetD16|hipMemsetD32|hipMemcpy2D|hipMemcpy3D)\s*\(")
ALLOWED_FUNCS = {"pscl_create"}


def strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", lambda m: re.sub(r"[^\n]", " ", m.group(0)), src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return re.sub(r'"(?:\\.|[^"\\])*"', '""', src)


def function_spans(src: str):
    """(name, start, end) of every top-level brace block that follows a function signature."""
    spans, depth, i, start, name = [], 0, 0, None, None
    sig = re.compile(r"([A-Za-z_]\w*)\s*\([^;{}]*\)\s*(?:const\s*)?(?:->\s*[\w:<>]+\s*)?$")
    while i < len(src):
        c = src[i]
        if c == "{":
            if depth == 0 or (depth == 1 and name is None and start is None):
                head = src[max(0, i - 400):i].rstrip()
                m = sig.search(head)
                if m and m.group(1) not in ("if", "for", "while", "switch", "catch"):
                    name, start = m.group(1), i
                    d, j = 0, i
                    while j < len(src):
                        if src[j] == "{":
                            d += 1
                        elif src[j] == "}":
                            d -= 1
                            if d == 0:
                                break
                        j += 1
                    spans.append((name, start, j))
                    i = j + 1
                    name, start = None, None
                    continue
            depth += 1
        elif c == "}":
            depth = max(0, depth - 1)
        i += 1
    return spans


def test_no_synchronous_device_writes_outside_create():
    offenders = []
    for f in sorted([*CSRC.glob("*.cpp"), *CSRC.glob("*.hip"), *CSRC.glob("*.h")]):
        src = strip_comments(f.read_text())
        spans = function_spans(src)
        for m in SYNC_CALLS.finditer(src):
            owner = next((n for n, a, b in spans if a <= m.start() <= b), "<file scope>")
            if owner not in ALLOWED_FUNCS:
                line = src.count("\n", 0, m.start()) + 1
                offenders.append(f"{f.name}:{line} {m.group(1)} in {owner}")
    assert not offenders, "synchronous device copies/fills outside pscl_create: " + "; ".join(offenders)


def test_scanner_finds_known_calls():
    """The scanner itself: pscl_create's uploads are found and attributed to it."""
    src = strip_comments((CSRC / "capi.cpp").read_text())
    spans = function_spans(src)
    owners = {next((n for n, a, b in spans if a <= m.start() <= b), None) for m in SYNC_CALLS.finditer(src)}
    assert owners == {"pscl_create"}
    fake = "int pscl_other(int x) {\n  if (x) { hipMemset(p, 0, 4); }\n  return 0;\n}\n"
    sp = function_spans(fake)
    assert [n for n, _, _ in sp] == ["pscl_other"]
