"""Golden-data test runner: the counterpart of the reference's QuESTTest
(``utilities/QuESTTest/QuESTCore.py:380-492`` for the case semantics,
``utilities/QuESTTest/__main__.py`` for the CLI).

Each case of ``tests/data/reference_golden.json`` (converted from the
reference's ``.test`` files by ``tools/import_reference_tests.py``) names an
API function, an initial state (``z`` zero, ``p`` plus, ``d`` debug, ``c``
custom amplitudes, ``b`` bit string; upper case = density matrix), the
function's arguments, and the expected outcome:

* ``P``  total probability (calcTotalProb),
* ``M``  calcProbOfOutcome(q, 0/1) for every qubit,
* ``S``  every amplitude (the full flattened state; the reference's runner
  compares only a corner of a density matrix, this one compares all of it),
* or the function's return value.

Tolerances are absolute for values of magnitude <= 1 and relative above
(the debug states reach |amp| ~ 12); fp64 runs use 1e-10 (the reference's
CLI default), fp32 builds need ~2e-4 (cos/sin of the data's 300-rad angles).

Runs on whatever backend and rank layout the process has (every rank runs
every case; distributed runs exercise the exchange paths with 3-qubit
registers spread over 2-4 ranks, like the reference's ``mpiexec -n 4``).

    python -m quest_amd.utils.golden [--filter hadamard] [--tol 1e-10] [--log out]
    python -m quest_amd.utils.golden --generate new.json   # expectations from this build
"""
from __future__ import annotations

import argparse
import json
import os
import sys

DEFAULT_DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests",
                            "data", "reference_golden.json")


def load_suites(path: str = DEFAULT_DATA) -> dict:
    with open(path) as f:
        return json.load(f)["suites"]


def _cx(v):
    return complex(v[0], v[1])


def _convert_args(func: str, args: list) -> list:
    out = []
    for a in args:
        if isinstance(a, list) and a and isinstance(a[0], list):  # list of complex
            out.append([_cx(x) for x in a])
        elif isinstance(a, list) and len(a) == 2 and func in ("compactUnitary", "controlledCompactUnitary") \
                and all(isinstance(x, float) for x in a):
            out.append(_cx(a))
        else:
            out.append(a)
    if func == "setAmps":  # (startInd, reals, imags, numAmps) with scalar amps in the data
        start, re, im, num = out
        out = [start, re if isinstance(re, list) else [re], im if isinstance(im, list) else [im], num]
    return out


def _make_register(capi, env, case):
    n = case["n"]
    q = capi.createDensityQureg(n, env) if case["density"] else capi.createQureg(n, env)
    init = case["init"].lower()
    if init == "z":
        capi.initZeroState(q)
    elif init == "p":
        capi.initPlusState(q)
    elif init == "d":
        capi.initStateDebug(q)
    elif init == "b":
        capi.initClassicalState(q, int(case["bits"], 2))
    elif init == "c":
        re = [a[0] for a in case["amps"]]
        im = [a[1] for a in case["amps"]]
        if case["density"]:
            capi.setDensityAmps(q, re, im)
        else:
            capi.setAmps(q, 0, re, im, len(re))
    else:
        raise ValueError(f"unknown initial state {case['init']}")
    return q


class Skip(Exception):
    pass


def run_case(capi, env, func: str, case: dict, tol: float) -> list[str]:
    """Run one case; returns a list of failure descriptions (empty = pass).
    Raises Skip when the register cannot be spread over this many ranks
    (fewer than 2 amplitudes per rank; E_TOO_MANY_QUBITS_FOR_RANKS)."""
    nsv = case["n"] * (2 if case["density"] else 1)
    if (1 << nsv) < 2 * env.numRanks:
        raise Skip()
    q = _make_register(capi, env, case)
    errs = []
    try:
        fn = getattr(capi, func)
        args = _convert_args(func, case["args"])
        if "returns" in case:
            got = fn(q, *args)
            want = case["returns"]
            if isinstance(want, list):
                if abs(complex(got) - _cx(want)) > tol * 1.5 * max(1.0, abs(_cx(want))):
                    errs.append(f"returned {got}, expected {_cx(want)}")
            elif isinstance(want, int) and not isinstance(want, bool) and func.startswith("getNum"):
                if got != want:
                    errs.append(f"returned {got}, expected {want}")
            elif abs(float(got) - float(want)) > tol * max(1.0, abs(float(want))):
                errs.append(f"returned {got}, expected {want}")
        else:
            fn(q, *args)
            exp = case["expect"]
            if "P" in exp:
                got = capi.calcTotalProb(q)
                if abs(got - exp["P"]) > tol * max(1.0, abs(exp["P"])):
                    errs.append(f"total prob {got} != {exp['P']}")
            if "M" in exp:
                for qb, (p0, p1) in enumerate(exp["M"]):
                    g0, g1 = capi.calcProbOfOutcome(q, qb, 0), capi.calcProbOfOutcome(q, qb, 1)
                    if abs(g0 - p0) > tol * max(1.0, abs(p0)) or abs(g1 - p1) > tol * max(1.0, abs(p1)):
                        errs.append(f"qubit {qb} probs ({g0}, {g1}) != ({p0}, {p1})")
            if "S" in exp:
                import numpy as np

                got = capi.getAmps(q, 0, q.numAmpsTotal)
                want = np.array([_cx(a) for a in exp["S"]])
                scale = np.maximum(1.0, np.abs(want))
                d = float(np.max(np.maximum(np.abs(got.real - want.real), np.abs(got.imag - want.imag)) / scale))
                if d > tol:
                    errs.append(f"state differs by {d:.3g}")
    finally:
        capi.destroyQureg(q, env)
    return errs


def observe_case(capi, env, func: str, case: dict) -> dict:
    """Run a case and return what this build produces, in the case's own
    schema ("returns" or "expect" with the case's P/M/S checks): the
    reference runner's golden-generation mode (QuESTCore.py:584-711)."""
    import numpy as np

    q = _make_register(capi, env, case)
    try:
        fn = getattr(capi, func)
        args = _convert_args(func, case["args"])
        if "returns" in case:
            got = fn(q, *args)
            if isinstance(got, complex):
                return {"returns": [got.real, got.imag]}
            return {"returns": got}
        fn(q, *args)
        exp = {}
        for chk in (case.get("checks") or "S"):
            if chk in "Pp":
                exp["P"] = capi.calcTotalProb(q)
            elif chk in "Mm":
                exp["M"] = [[capi.calcProbOfOutcome(q, b, 0), capi.calcProbOfOutcome(q, b, 1)]
                            for b in range(case["n"])]
            elif chk in "Ss":
                amps = capi.getAmps(q, 0, q.numAmpsTotal)
                exp["S"] = [[float(a.real), float(a.imag)] for a in np.asarray(amps)]
        return {"expect": exp}
    finally:
        capi.destroyQureg(q, env)


def generate(out_path: str, env=None, path: str = DEFAULT_DATA, filt: str | None = None) -> int:
    """Write a copy of the golden data whose expectations come from this
    build (regression baselines for new cases or other precisions)."""
    from ..ops import capi

    with open(path) as f:
        data = json.load(f)
    own_env = env is None
    if own_env:
        env = capi.createQuESTEnv()
    n = 0
    try:
        for name, suite in data["suites"].items():
            if filt and filt not in name:
                continue
            for case in suite["cases"]:
                nsv = case["n"] * (2 if case["density"] else 1)
                if (1 << nsv) < 2 * env.numRanks:
                    continue
                obs = observe_case(capi, env, suite["function"], case)
                case.pop("returns", None)
                case.pop("expect", None)
                case.update(obs)
                n += 1
        data["source"] = "generated by quest_amd.utils.golden --generate"
        if env.rank == 0:
            with open(out_path, "w") as f:
                json.dump(data, f, separators=(",", ":"))
    finally:
        if own_env:
            capi.destroyQuESTEnv(env)
    return n


def run_all(env=None, filt: str | None = None, tol: float = 1e-10, path: str = DEFAULT_DATA,
            verbose: bool = False) -> tuple[int, list[str]]:
    from ..ops import capi

    own_env = env is None
    if own_env:
        env = capi.createQuESTEnv()
    passed = 0
    failures = []
    try:
        for name, suite in load_suites(path).items():
            if filt and filt not in name:
                continue
            func = suite["function"]
            for i, case in enumerate(suite["cases"]):
                try:
                    errs = run_case(capi, env, func, case, tol)
                except Skip:
                    continue
                if errs:
                    failures.append(f"{name}[{i}] {case['init']}-{case['checks']} {case['args']}: {'; '.join(errs)}")
                else:
                    passed += 1
                if verbose:
                    print(("F " if errs else ". ") + f"{name}[{i}]", flush=True)
    finally:
        if own_env:
            capi.destroyQuESTEnv(env)
    return passed, failures


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--filter", default=None, help="substring of the suite path")
    ap.add_argument("--tol", type=float, default=1e-10)
    ap.add_argument("--data", default=DEFAULT_DATA)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--generate", metavar="OUT", default=None,
                    help="write the data with expectations produced by this build to OUT")
    ap.add_argument("--log", metavar="FILE", default=None, help="also write results to FILE.<rank>")
    args = ap.parse_args(argv)
    from ..ops import capi

    env = capi.createQuESTEnv()
    if args.generate:
        n = generate(args.generate, env, args.data, args.filter)
        if env.rank == 0:
            print(f"generated {n} cases -> {args.generate}")
        capi.destroyQuESTEnv(env)
        return 0
    passed, failures = run_all(env, args.filter, args.tol, args.data, args.verbose)
    lines = [f"FAIL {f}" for f in failures] + [f"{passed} passed, {len(failures)} failed"]
    if env.rank == 0:
        print("\n".join(lines))
    if args.log:
        with open(f"{args.log}.{env.rank}", "w") as f:
            f.write("\n".join(lines) + "\n")
    capi.destroyQuESTEnv(env)
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
