class NotEnoughParticles(Exception):
    """pyabc/transition/exceptions.py:1-2."""
