"""birdnest.audio_amd -- MI355X-native FLAC frame decode behind BirdNest.Audio's surface."""
