import sys

from .cluster_bench import main

sys.exit(main())
