"""Host side of the gfx950 kernel library (include/ducosy_hip.h)."""
