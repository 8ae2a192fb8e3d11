"""csmom -- MI355X-native engine for the cross-sectional momentum backtest hot path of
AkshayJha22/Cross-Sectional-Momentum-Strategy-Replication-Backtesting-Framework.

Import it as ``csmom`` (the repo-root ``csmom.py`` aliases this directory, whose name is not
a Python identifier).  Public API (reference file:line it replaces):

  compute_monthly_momentum_from_daily   src/features.py:5-57       (GPU)
  compute_monthly_turnover              src/features.py:60-107     (host; unused by the path)
  assign_deciles_per_date               run_demo.py:18-29          (GPU)
  monthly_replication                   run_demo.py:31-79          (GPU + host summary)
  sharpe / ensure_dir / save_plot       src/utils.py:5-21          (host)
  fetch_daily / normalize_daily_columns src/data_io.py:23-73,131-180 (host, cached CSVs only)
  Engine                                dense device pipeline (bench / multi-GPU)
  Engine.portfolio / Engine.bootstrap   K-overlap, value weights, turnover, costs, bootstrap
                                        (beyond run_demo.py:49-67)
  SweepRunner                           (J, K) grids over panels / bootstrap panels (C3, C5)
  Engine.turnover_features              src/features.py:60-107 on the device (bit-exact)
  momentum_volume_double_sort           LeSw00 10 x 3 momentum x turnover sort
"""
from ._lib import ABSENT_BITS, CsmError, CsmUnavailable, lib_path, load_library
from .engine import Engine, PipelineOut, PortfolioOut, absent_tensor, is_absent, quantile_table
from .data import fetch_daily, load_daily_panel, normalize_daily_columns
from .features import compute_monthly_momentum_from_daily, compute_monthly_turnover, get_engine
from .lesw import DoubleSortResult, momentum_volume_double_sort
from .panel import DensePanel, from_long, month_offsets, monthly_frame
from .replication import ReplicationResult, assign_deciles_per_date, monthly_replication
from .sweep import SUMMARY_FIELDS, SweepConfig, SweepRunner, strategy_grid
from .utils import ensure_dir, save_plot, sharpe

__all__ = [
    "ABSENT_BITS", "CsmError", "CsmUnavailable", "lib_path", "load_library", "Engine",
    "PipelineOut", "PortfolioOut", "SweepConfig", "SweepRunner", "SUMMARY_FIELDS",
    "strategy_grid", "DoubleSortResult", "momentum_volume_double_sort", "fetch_daily", "load_daily_panel", "normalize_daily_columns",
    "absent_tensor", "is_absent", "quantile_table",
    "compute_monthly_momentum_from_daily", "compute_monthly_turnover", "get_engine",
    "DensePanel", "from_long", "month_offsets", "monthly_frame", "ReplicationResult",
    "assign_deciles_per_date", "monthly_replication", "ensure_dir", "save_plot", "sharpe",
]
