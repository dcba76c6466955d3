"""e2ep_amd — MI355X-native runtime for the ParkingModel hot path (HIP kernels + C-ABI)."""
