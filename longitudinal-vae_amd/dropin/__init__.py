"""Drop-in modules for the reference's flat import surface.

Put this directory ahead of the reference checkout on ``sys.path`` and the
reference's ``training.py`` / ``validation.py`` / ``model_test.py`` imports
(``from elbo_functions import ...``, ``from kernel_gen import ...``, ``from utils import ...``)
resolve to the MI355X implementation in ``lvae_amd``.
"""
