"""Mirror of src/examples/botnet/botnet_augmented_constraints.py."""
from .botnet_constraints import BotnetAugmentedConstraints  # noqa: F401
