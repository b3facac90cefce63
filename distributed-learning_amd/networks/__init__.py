"""Model families of the reference's consensus workloads (reference networks/)."""
from .ann_model import ANNModel  # noqa: F401
from .logreg_model_titanic import LogRegTitanic  # noqa: F401
