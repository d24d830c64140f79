#!/usr/bin/env python3
"""Convert the reference's golden ``.test`` data files into one JSON fixture.

The reference keeps its unit-test expectations as text files
(``tests/unit/**/*.test``; grammar documented by its runner,
``utilities/QuESTTest/QuESTCore.py:380-492``):

    # <function>
    <number of cases>
    <init>-<checks> <nQubits> [<initial amps or bit string>] <args...>
    <expected data: P total probability, M per-qubit (p0 p1), S amplitudes,
     or a single returned value>

Only the data is taken (files holding Python code are skipped; their checks
are re-written as pytest tests in tests/test_reference_suite.py).  The
output, ``tests/data/reference_golden.json``, is what the test suite reads,
so the tests need nothing from the reference at run time.

    python tools/import_reference_tests.py /root/reference/tests
"""
from __future__ import annotations

import json
import os
import re
import sys

RETURNING = {"calcProbOfOutcome", "calcTotalProb", "calcPurity", "getAmp", "getRealAmp", "getImagAmp",
             "getProbAmp", "getDensityAmp", "getNumAmps", "getNumQubits"}

_CPLX = re.compile(r"\(\s*([-+0-9.eE]+)\s*,\s*([-+0-9.eE]+)\s*\)")


def parse_value(tok: str):
    """One argument token -> JSON value: number, [re, im], list of numbers,
    or list of [re, im]."""
    tok = tok.strip()
    if tok.startswith("["):
        if "(" in tok:
            return [[float(a), float(b)] for a, b in _CPLX.findall(tok)]
        body = tok.strip("[]").strip().rstrip(",")
        return [float(x) if any(c in x for c in ".eE") else int(x) for x in body.split(",") if x.strip()]
    if tok.startswith("("):
        m = _CPLX.match(tok)
        return [float(m.group(1)), float(m.group(2))]
    if any(c in tok for c in ".eE") or tok.lower() in ("nan", "inf"):
        return float(tok)
    return int(tok)


def split_args(s: str):
    """Whitespace split that keeps bracketed groups together."""
    out, cur, depth = [], "", 0
    for ch in s:
        if ch in "[(":
            depth += 1
        elif ch in "])":
            depth = max(0, depth - 1)
        if ch.isspace() and depth == 0:
            if cur:
                out.append(cur)
                cur = ""
        else:
            cur += ch
    if cur:
        out.append(cur)
    return out


def parse_file(path: str):
    with open(path) as f:
        raw = [ln.rstrip("\n") for ln in f]
    if raw and raw[0].startswith("# Python"):
        return None
    lines = [ln.strip() for ln in raw if ln.strip() and not ln.strip().startswith("#")]
    func = raw[0].lstrip("# ").strip()
    n_cases = int(lines[0])
    pos = 1
    cases = []
    for _ in range(n_cases):
        head = split_args(lines[pos])
        pos += 1
        spec, nbits = head[0], int(head[1])
        args = head[2:]
        init, _, checks = spec.partition("-")
        checks = checks.strip()
        if nbits == 0:
            continue
        density = init.isupper()
        case = {"init": init, "density": density, "n": nbits, "checks": checks}
        if init.lower() == "c":
            case["amps"] = parse_value(args[0])
            args = args[1:]
        elif init.lower() == "b":
            case["bits"] = args[0]
            args = args[1:]
        case["args"] = [parse_value(a) for a in args]
        if func in RETURNING:
            v = lines[pos]
            pos += 1
            case["returns"] = parse_value(v)
        else:
            exp = {}
            for chk in (checks or "S"):
                if chk in "Pp":
                    exp["P"] = float(lines[pos])
                    pos += 1
                elif chk in "Mm":
                    exp["M"] = [[float(x) for x in lines[pos + q].split()] for q in range(nbits)]
                    pos += nbits
                elif chk in "Ss":
                    cnt = 1 << (2 * nbits if density else nbits)
                    exp["S"] = [parse_value(lines[pos + i]) for i in range(cnt)]
                    pos += cnt
            case["expect"] = exp
        cases.append(case)
    return func, cases


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/tests"
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "data", "reference_golden.json")
    suites = {}
    for root, _, files in sorted(os.walk(src)):
        for fn in sorted(files):
            if not fn.endswith(".test"):
                continue
            path = os.path.join(root, fn)
            got = parse_file(path)
            if got is None:
                continue
            func, cases = got
            rel = os.path.relpath(path, src)
            suites[rel] = {"function": func, "cases": cases}
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        json.dump({"source": "reference tests/**/*.test (golden data only)", "suites": suites}, f,
                  separators=(",", ":"))
    total = sum(len(s["cases"]) for s in suites.values())
    print(f"{len(suites)} files, {total} cases -> {dst}")


if __name__ == "__main__":
    main()
