#!/usr/bin/env python3
"""Gang-placement validation on one node (one rank per GPU); see
``yoda_scheduler_amd/parallel/validate_gangs.py``.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        scripts/validate_gangs.py --k 4 --load-pairs 0-1,2-3
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from yoda_scheduler_amd.parallel.validate_gangs import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
