"""dopamine_amd agents."""
