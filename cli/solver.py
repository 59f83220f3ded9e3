"""Alias of distilp_amd.cli.solver (reference console script `solver` = cli.solver:main)."""

import sys

from distilp_amd.cli.solver import (  # noqa: F401
    load_device_profile,
    load_devices_and_model,
    load_from_profile_folder,
    load_model_profile,
    main,
)

if __name__ == "__main__":
    sys.exit(main())
