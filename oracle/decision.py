"""Restatement of the reference's per-frame movement / output decision.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Given the external-contour
count of every frame -- the only output of the hot path the decision reads --
return the source frame indices the reference writes, in write order:

* find_movement  fm.py:665-700: movement = count > 0; movement_counter += count
  (one per contour, fm.py:694), reset to 0 on a frame without contours
  (fm.py:697-698); movement_decay decremented first (fm.py:672);
* decide_output  fm.py:549-589: write when movement_counter >= min_movement_frames
  or movement_decay > 0; on a movement frame first flush the pre-motion cache
  (fm.py:558-570) and re-arm the decay to cache_frames; otherwise push the
  frame into deque(maxlen=cache_frames) (fm.py:415, 588).
"""
from collections import deque


def written_indices(counts, fps: int = 30, min_time: float = 0.5, cache_time: float = 1.0, current_only: bool = False):
    """current_only: only the frames written as the current frame -- the ones decide_output also
    runs find_objects on (fm.py:571-575); flushed cache frames are left out."""
    cache_frames = int(cache_time * fps)
    min_frames = int(min_time * fps)
    cache = deque(maxlen=cache_frames)
    counter, decay, out = 0, 0, []
    for i, c in enumerate(counts):
        movement = False
        decay -= 1 if decay > 0 else 0
        if c > 0:
            counter += int(c)
            movement = True
        if not movement:
            counter = 0
        if counter >= min_frames or decay > 0:
            if movement:
                decay = cache_frames
                if not current_only:
                    out.extend(cache)
                cache.clear()
            out.append(i)
        else:
            cache.append(i)
    return out
