"""MI355X-native ACC-UNet (gfx950 HIP kernels behind the reference nn.Module API)."""
