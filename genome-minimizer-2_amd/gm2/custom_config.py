"""ExperimentConfig — field names and defaults of src/genome_minimizer_2/utils/custom_config.py:13-54
(batch 32, lr 1e-3, max_norm 1.0, StepLR 20 / 0.5, split 0.3 / 0.3333 / seed 12345). The interactive
and JSON-driven `--mode experiment` plumbing of that file is out of scope."""
from dataclasses import asdict, dataclass, fields


@dataclass
class ExperimentConfig:
    hidden_dim: int = 512
    latent_dim: int = 32
    n_epochs: int = 1
    batch_size: int = 32
    learning_rate: float = 1e-3
    max_norm: float = 1.0
    lambda_l1: float = 0.01
    min_beta: float = 0.0
    max_beta: float = 1.0
    gamma_start: float = 1.0
    gamma_end: float = 0.1
    weight: float = 1.0
    trainer_version: str = "v2"
    scheduler_step_size: int = 20
    scheduler_gamma: float = 0.5
    test_size: float = 0.3
    val_ratio: float = 0.3333
    random_state: int = 12345
    experiment_name: str = "experiment"
    save_model: bool = True
    generate_plots: bool = True
    calculate_metrics: bool = True
    explore_latent_space: bool = True

    def update_from_dict(self, d):
        names = {f.name for f in fields(self)}
        for k, v in d.items():
            if k in names:
                setattr(self, k, v)
        return self

    def to_dict(self):
        return asdict(self)
