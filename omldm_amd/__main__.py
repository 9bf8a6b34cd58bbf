import sys

from omldm_amd.cli import main

sys.exit(main())
