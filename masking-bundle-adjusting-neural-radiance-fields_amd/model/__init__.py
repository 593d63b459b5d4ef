"""Models (the reference ships only `planar`)."""
