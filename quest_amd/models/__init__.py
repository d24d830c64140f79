"""Circuit families (see circuits.py)."""
from .circuits import (  # noqa: F401
    Circuit,
    Gate,
    bernstein_vazirani,
    fork_benchmark,
    fork_circuit,
    load_api_circuit,
    ghz,
    qft,
    random_layered,
    random_mixed,
)
