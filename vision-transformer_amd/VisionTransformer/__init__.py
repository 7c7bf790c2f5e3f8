"""MI355X-native drop-in for the reference VisionTransformer package (config, transformer, vit)."""
