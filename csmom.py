"""Import alias: ``import csmom`` loads the package directory
``cross-sectional-momentum-strategy-replication-backtesting-framework_amd/`` (its name is
not a Python identifier)."""
import importlib.util
import pathlib
import sys

_DIR = pathlib.Path(__file__).resolve().with_name(
    "cross-sectional-momentum-strategy-replication-backtesting-framework_amd")
_spec = importlib.util.spec_from_file_location(
    "csmom", _DIR / "__init__.py", submodule_search_locations=[str(_DIR)])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["csmom"] = _mod
_spec.loader.exec_module(_mod)
