"""MI355X-native batched PianoWithShadowHands environment."""
