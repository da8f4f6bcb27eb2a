// Event.h — input event of the FARMS_Flow path.
//
// Same public interface as the reference's Event (/root/reference/include/
// Event.h:14-45): x, y, polarity and a double time stamp, with setters that
// return true and plain getters.  Kept for drop-in source compatibility of code
// that builds Event objects around vFlowManager.
#ifndef FARMS_HOST_EVENT_H
#define FARMS_HOST_EVENT_H

class Event {
public:
    Event(int x, int y, double t, int p);
    Event();

    bool setX(int v);
    bool setY(int v);
    bool setStamp(double v);
    bool setPolarity(int v);

    int getX() const;
    int getY() const;
    double getStamp() const;
    int getPolarity() const;

private:
    int x_;
    int y_;
    int pol_;
    double t_;
};

#endif
