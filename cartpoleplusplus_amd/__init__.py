"""MI355X-native batched cartpole++."""
