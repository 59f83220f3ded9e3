"""distilp_amd — MI355X-native HALDA solver behind the distilp.solver API.

The fixed-k HALDA MILP and its k-sweep (reference: firstbatchxyz/distilp,
src/distilp/solver/halda_p_solver.py) run on AMD Instinct MI355X (gfx950)
through libhalda, a HIP library reached over a plain C ABI (include/halda.h).
"""

__version__ = "0.1.0"
