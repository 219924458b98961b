"""MI355X-native ABCD-VAE modules (mirrors the reference's ``modules`` package)."""
