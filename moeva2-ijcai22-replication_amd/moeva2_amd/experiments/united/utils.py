"""project_name -> Constraints class registry (mirror of src/experiments/united/utils.py:12-26).
The SAT (Gurobi) registry is out of scope."""
from ...examples.botnet.botnet_constraints import BotnetAugmentedConstraints, BotnetConstraints
from ...examples.lcld.lcld_augmented_constraints import LcldAugmentedConstraints
from ...examples.lcld.lcld_constraints import LcldConstraints

STR_TO_CONSTRAINTS_CLASS = {
    "lcld": LcldConstraints,
    "botnet": BotnetConstraints,
    "lcld_augmented": LcldAugmentedConstraints,
    "botnet_augmented": BotnetAugmentedConstraints,
}


def get_constraints_from_str(project_name: str):
    return STR_TO_CONSTRAINTS_CLASS[project_name]
