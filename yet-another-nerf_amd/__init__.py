"""yanerf_amd: MI355X-native volumetric-rendering hot path for yet-another-nerf."""
