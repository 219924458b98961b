# coding: utf-8
"""ABCD-VAE/encode_logit.py: same as encode.py but writes the logits."""
import encode

if __name__ == "__main__":
    encode.main(output="logits")
