"""Drop-in for lib/in_development/models_bayes.py (served by ude_amd.bayes)."""
from ude_amd.bayes import Dense_Variational, Bayes_Fp, Bayes_Fa, Bayes_FaFp  # noqa: F401
