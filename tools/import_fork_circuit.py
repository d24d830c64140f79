#!/usr/bin/env python3
"""Extract the fork's 30-qubit benchmark circuit (the reference's
``tutorial_example.c:29-518``: 490 gate calls, then 30 calcProbOfOutcome and
10 getAmp) into a plain text circuit file, one gate per line:

    <function> <int args...> [<angle>]

The output, ``examples/data/fork_circuit_30q.txt``, is read by
``quest_amd.models.circuits.fork_circuit()`` and by
``examples/fork_benchmark.c``; nothing is read from the reference at run
time.

    python tools/import_fork_circuit.py [/root/reference/tutorial_example.c]
"""
import os
import re
import sys

CALL = re.compile(r"^\s*([A-Za-z]+)\(q,\s*([^)]*)\);")


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/tutorial_example.c"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(root, "examples", "data", "fork_circuit_30q.txt")
    gates = []
    with open(src) as f:
        for line in f:
            m = CALL.match(line)
            if not m or m.group(1) in ("destroyQureg", "calcProbOfOutcome", "getAmp"):
                continue
            args = [a.strip() for a in m.group(2).split(",")]
            gates.append((m.group(1), args))
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        f.write("# fork benchmark circuit: 30 qubits, %d gates (tutorial_example.c:29-518)\n" % len(gates))
        for name, args in gates:
            f.write(name + " " + " ".join(args) + "\n")
    print(f"{len(gates)} gates -> {dst}")


if __name__ == "__main__":
    main()
