"""genome-minimizer-2 · MI355X: the VAE train + sample hot path of ucl-cssb/genome-minimizer-2,
re-built on hand-written gfx950 HIP kernels (libgm2.so) behind the reference's Python interface.

Modules mirror the reference layout they replace:
  model.py            <- src/genome_minimizer_2/training/model.py
  loss_components.py  <- src/genome_minimizer_2/training/training/loss_components.py
  trainer.py          <- src/genome_minimizer_2/training/training/trainer.py
  custom_config.py    <- src/genome_minimizer_2/utils/custom_config.py (ExperimentConfig)
  experiments.py      <- src/genome_minimizer_2/utils/experiments.py (presets, runner)
  extras.py           <- src/genome_minimizer_2/utils/extras.py (load_model, sample_from_model, ...)
  data.py             <- explore_data/data_exploration.py:load_and_validate_data + DataLoader semantics
  native.py           :  ctypes binding of libgm2.so (include/gm2.h)
"""
from .native import GM2_BF16, GM2_F32  # noqa: F401

__version__ = "0.1.0"
