"""elbo_functions.py surface (reference elbo_functions.py:8-307) backed by lvae_amd (HIP)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lvae_amd.elbo import KL_closed, minibatch_KLD_upper_bound, minibatch_KLD_upper_bound_iter  # noqa: E402,F401
from lvae_amd.gpapprox import deviance_upper_bound, elbo  # noqa: E402,F401

__all__ = ["KL_closed", "elbo", "deviance_upper_bound", "minibatch_KLD_upper_bound", "minibatch_KLD_upper_bound_iter"]
