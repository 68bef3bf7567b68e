from .trainer import MlpTrainer, StepStats  # noqa: F401
