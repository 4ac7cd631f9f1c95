"""Host-side mirror of the reference recordio package surface."""
