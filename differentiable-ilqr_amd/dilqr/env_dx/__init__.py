"""Dynamics models of the reference (env_dx/), evaluated by the HIP library."""
