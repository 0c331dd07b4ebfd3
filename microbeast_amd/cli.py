"""Entry point: ``python microbeast.py [--exp_name NAME] [--test] [--flag value ...]``.

Reference: parser.py + microbeast.py:267-278 (``main()`` -> ``test()`` or
``train(args.exp_name)``).
"""
from __future__ import annotations

import sys

from .config import parse_flags


def main(argv=None) -> int:
    flags = parse_flags(argv)
    if flags.test:
        from .evaluate import evaluate

        evaluate(flags)
    else:
        from .train import train

        train(flags)
    return 0


if __name__ == "__main__":
    sys.exit(main())
