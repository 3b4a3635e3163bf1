"""Frame loops over `Scene.render` (reference `sightpy/animation.py:6-54`)."""
from pathlib import Path

import numpy as np

__all__ = ["create_animation", "create_animation_using_opencv"]


def create_animation(scene, samples_per_pixel, fps, start_time, final_time, update_scene, name):
    number_of_frames = int(fps * (final_time - start_time))
    dt = (final_time - start_time) / number_of_frames
    t = start_time
    Path("./frames").mkdir(exist_ok=True)
    for i in range(number_of_frames):
        update_scene(scene, t)
        img = scene.render(samples_per_pixel)
        t += dt
        img.save("frames/" + name + "_" + str(i) + ".png")


def create_animation_using_opencv(scene, samples_per_pixel, fps, start_time, final_time, update_scene, name):
    import cv2

    number_of_frames = int(fps * (final_time - start_time))
    dt = (final_time - start_time) / number_of_frames
    t = start_time
    dims = (scene.camera.screen_width, scene.camera.screen_height)
    video = cv2.VideoWriter(name, cv2.VideoWriter_fourcc("M", "J", "P", "G"), fps, dims)
    for i in range(number_of_frames):
        update_scene(scene, t)
        frame = scene.render(samples_per_pixel)
        video.write(cv2.cvtColor(np.array(frame), cv2.COLOR_RGB2BGR))
        t += dt
    video.release()
