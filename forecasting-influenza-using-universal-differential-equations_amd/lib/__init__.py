"""Drop-in for the reference's ``lib`` package (lib/models.py, lib/train_functions.py,
lib/VAE.py, lib/utils.py, lib/Metrics.py, lib/in_development/models_bayes.py).

With ``<this package dir>`` on ``sys.path`` (importing the package does that),
``import lib.models`` / ``from lib.VAE import VAE`` resolve here, and the ODE
classes run their RK4 solves on the fused gfx950 kernel.
"""
