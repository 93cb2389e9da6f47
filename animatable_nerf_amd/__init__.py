"""MI355X-native Animatable-NeRF volume-rendering hot path."""
