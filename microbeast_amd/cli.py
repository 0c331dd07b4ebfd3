"""Entry point: ``python microbeast.py [--exp_name NAME] [--test] [--flag value ...]``.

Reference: parser.py + microbeast.py:267-278 (``main()`` -> ``test()`` or
``train(args.exp_name)``).

``--nproc_per_node N`` (N > 1) outside torchrun launches N data-parallel ranks
(one per GPU) as a child ``torch.distributed.run`` and returns its exit code;
the experiment-name prompt happens once, here, and the name is passed on.
"""
from __future__ import annotations

import os
import sys

from .config import parse_flags


def main(argv=None) -> int:
    flags = parse_flags(argv)
    if flags.nproc_per_node > 1 and "WORLD_SIZE" not in os.environ and not flags.test:
        from .parallel.launch import relaunch

        child = list(sys.argv[1:] if argv is None else argv) + ["--exp_name", flags.exp_name]
        return relaunch(flags.nproc_per_node, child, module="microbeast_amd",
                        shared_gpu=flags.device == "cpu")  # CPU DP ranks need no GPU
    if flags.test:
        from .evaluate import evaluate

        try:
            evaluate(flags)
        except FileNotFoundError as e:  # no checkpoint: fail, do not score random weights
            print(f"microbeast: {e}", file=sys.stderr)
            return 2
    else:
        from .train import train

        train(flags)
    return 0


if __name__ == "__main__":
    sys.exit(main())
