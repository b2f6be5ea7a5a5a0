"""Rank-side entry of ``cloudtik_amd.runner.run``: load the function this job's driver
serialized into WORKDIR, call it, write ``result_<RANK>.pkl``."""
import os
import sys


def main():
    import cloudpickle
    work = sys.argv[1]
    with open(os.path.join(work, "func.pkl"), "rb") as f:
        fn, args, kwargs = cloudpickle.load(f)
    result = fn(*args, **kwargs)
    rank = int(os.environ.get("RANK", "0"))
    tmp = os.path.join(work, f".result_{rank}.pkl")
    with open(tmp, "wb") as f:
        cloudpickle.dump(result, f)
    os.replace(tmp, os.path.join(work, f"result_{rank}.pkl"))


if __name__ == "__main__":
    main()
