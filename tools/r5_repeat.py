"""Run a pytest selection several times in ONE process (debugging a failure
that depends on what earlier tests left behind).

    python tools/r5_repeat.py REPS -- <pytest args>
"""
import sys

import pytest


def main():
    reps = int(sys.argv[1])
    args = sys.argv[sys.argv.index("--") + 1:]
    rcs = []
    for i in range(reps):
        rc = pytest.main(list(args))
        rcs.append(int(rc))
        print(f"== repetition {i}: rc {int(rc)}", flush=True)
        if int(rc) not in (0, 1):
            break
    print("rcs", rcs, flush=True)


if __name__ == "__main__":
    main()
