# coding: utf-8
"""ABCD-VAE/encode_features.py: same as encode.py but writes the features."""
import encode

if __name__ == "__main__":
    encode.main(output="features")
