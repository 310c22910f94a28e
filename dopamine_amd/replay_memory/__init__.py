"""Device-resident replay memories with Dopamine's out-of-graph API."""
