import sys
