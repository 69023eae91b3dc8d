"""birdnest -- namespace for the MI355X-native BirdNest.Audio FLAC decode path."""
